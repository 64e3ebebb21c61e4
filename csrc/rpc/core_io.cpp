#include "rpc/core_io.h"
#include "consensus/params.h"
#include "keys/key.h"
#include "rpc/server.h"
#include "script/interpreter.h"
#include "script/standard.h"
#include "util/strencodings.h"

namespace bcp {

bool DecodeHexTx(CMutableTransaction& tx, const std::string& strHexTx) {
    if (!IsHex(strHexTx)) return false;
    std::vector<unsigned char> data = ParseHex(strHexTx);
    try {
        SpanReader r(data.data(), data.size());
        r >> tx;
        return r.empty();
    } catch (const std::exception&) {
        return false;
    }
}

bool DecodeHexBlk(CBlock& block, const std::string& strHexBlk, bool fLegacyFormat) {
    if (!IsHex(strHexBlk)) return false;
    std::vector<unsigned char> data = ParseHex(strHexBlk);
    try {
        SpanReader r(data.data(), data.size(), SER_NETWORK, PROTOCOL_VERSION | (fLegacyFormat ? SERIALIZE_BLOCK_LEGACY : 0));
        r >> block;
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

bool DecodeHexBlockHeader(CBlockHeader& header, const std::string& hex, bool fLegacyFormat) {
    if (!IsHex(hex)) return false;
    std::vector<unsigned char> data = ParseHex(hex);
    try {
        SpanReader r(data.data(), data.size(), SER_NETWORK, PROTOCOL_VERSION | (fLegacyFormat ? SERIALIZE_BLOCK_LEGACY : 0));
        r >> header;
    } catch (const std::exception&) {
        return false;
    }
    return true;
}

std::string EncodeHexTx(const CTransaction& tx) { return HexStr(SerializeToBytes(tx)); }
std::string EncodeHexBlock(const CBlock& block, bool fLegacyFormat) {
    return HexStr(SerializeToBytes(block, SER_NETWORK, PROTOCOL_VERSION | (fLegacyFormat ? SERIALIZE_BLOCK_LEGACY : 0)));
}

uint256 ParseHashStr(const std::string& str, const std::string& name) {
    if (!IsHex(str) || str.size() != 64) throw std::runtime_error(name + " must be hexadecimal string (not '" + str + "')");
    return uint256S(str);
}

int ParseSighashString(const std::string& s) {
    static const std::pair<const char*, int> kMap[] = {
        {"ALL", SIGHASH_ALL},
        {"ALL|ANYONECANPAY", SIGHASH_ALL | SIGHASH_ANYONECANPAY},
        {"ALL|FORKID", SIGHASH_ALL | SIGHASH_FORKID},
        {"ALL|FORKID|ANYONECANPAY", SIGHASH_ALL | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
        {"NONE", SIGHASH_NONE},
        {"NONE|ANYONECANPAY", SIGHASH_NONE | SIGHASH_ANYONECANPAY},
        {"NONE|FORKID", SIGHASH_NONE | SIGHASH_FORKID},
        {"NONE|FORKID|ANYONECANPAY", SIGHASH_NONE | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
        {"SINGLE", SIGHASH_SINGLE},
        {"SINGLE|ANYONECANPAY", SIGHASH_SINGLE | SIGHASH_ANYONECANPAY},
        {"SINGLE|FORKID", SIGHASH_SINGLE | SIGHASH_FORKID},
        {"SINGLE|FORKID|ANYONECANPAY", SIGHASH_SINGLE | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
    };
    for (const auto& kv : kMap)
        if (s == kv.first) return kv.second;
    throw JSONRPCException{JSONRPCError(RPC_INVALID_PARAMETER, "Invalid sighash param")};
}

std::string FormatScript(const CScript& script) {
    std::string ret;
    CScript::const_iterator it = script.begin();
    opcodetype op;
    while (it != script.end()) {
        CScript::const_iterator it2 = it;
        std::vector<unsigned char> vch;
        if (script.GetOp(it, op, vch)) {
            if (op == OP_0) {
                ret += "0 ";
                continue;
            }
            if ((op >= OP_1 && op <= OP_16) || op == OP_1NEGATE) {
                ret += strprintf("%i ", (int)op - (int)OP_1NEGATE - 1);
                continue;
            }
            if (op >= OP_NOP && op <= OP_NOP10) {
                std::string str(GetOpName(op));
                if (str.substr(0, 3) == std::string("OP_")) {
                    ret += str.substr(3, std::string::npos) + " ";
                    continue;
                }
            }
            if (vch.size() > 0) ret += strprintf("0x%s 0x%s ", HexStr(it2, it - vch.size()).c_str(), HexStr(it - vch.size(), it).c_str());
            else ret += strprintf("0x%s ", HexStr(it2, it).c_str());
            continue;
        }
        ret += strprintf("0x%s ", HexStr(it2, script.end()).c_str());
        break;
    }
    return ret.substr(0, ret.size() ? ret.size() - 1 : 0);
}

void ScriptPubKeyToUniv(const CScript& scriptPubKey, UniValue& out, bool fIncludeHex, const CChainParams& params) {
    txnouttype type;
    std::vector<CTxDestination> addresses;
    int nRequired;
    out.pushKV("asm", ScriptToAsmStr(scriptPubKey));
    if (fIncludeHex) out.pushKV("hex", HexStr(scriptPubKey.begin(), scriptPubKey.end()));
    if (!ExtractDestinations(scriptPubKey, type, addresses, nRequired)) {
        out.pushKV("type", GetTxnOutputType(type));
        return;
    }
    out.pushKV("reqSigs", nRequired);
    out.pushKV("type", GetTxnOutputType(type));
    UniValue a(UniValue::VARR);
    for (const CTxDestination& addr : addresses) a.push_back(EncodeDestination(addr, params));
    out.pushKV("addresses", a);
}

void TxToUniv(const CTransaction& tx, const uint256& hashBlock, UniValue& entry, const CChainParams& params,
              bool fRpcSize) {
    entry.pushKV("txid", tx.GetHash().GetHex());
    entry.pushKV("hash", tx.GetHash().GetHex());
    entry.pushKV("version", tx.nVersion);
    if (fRpcSize) entry.pushKV("size", (int)tx.GetTotalSize());
    entry.pushKV("locktime", (int64_t)tx.nLockTime);
    UniValue vin(UniValue::VARR);
    for (const CTxIn& txin : tx.vin) {
        UniValue in(UniValue::VOBJ);
        if (tx.IsCoinBase()) {
            in.pushKV("coinbase", HexStr(txin.scriptSig.begin(), txin.scriptSig.end()));
        } else {
            in.pushKV("txid", txin.prevout.hash.GetHex());
            in.pushKV("vout", (int64_t)txin.prevout.n);
            UniValue o(UniValue::VOBJ);
            o.pushKV("asm", ScriptToAsmStr(txin.scriptSig, true));
            o.pushKV("hex", HexStr(txin.scriptSig.begin(), txin.scriptSig.end()));
            in.pushKV("scriptSig", o);
        }
        in.pushKV("sequence", (int64_t)txin.nSequence);
        vin.push_back(in);
    }
    entry.pushKV("vin", vin);
    UniValue vout(UniValue::VARR);
    for (unsigned i = 0; i < tx.vout.size(); i++) {
        const CTxOut& txout = tx.vout[i];
        UniValue out(UniValue::VOBJ);
        out.pushKV("value", ValueFromAmount(txout.nValue));
        out.pushKV("n", (int64_t)i);
        UniValue o(UniValue::VOBJ);
        ScriptPubKeyToUniv(txout.scriptPubKey, o, true, params);
        out.pushKV("scriptPubKey", o);
        vout.push_back(out);
    }
    entry.pushKV("vout", vout);
    if (!hashBlock.IsNull()) entry.pushKV("blockhash", hashBlock.GetHex());
    entry.pushKV("hex", EncodeHexTx(tx));
}

double GetDifficultyFromBits(uint32_t nBits) {
    int nShift = (nBits >> 24) & 0xff;
    double dDiff = (double)0x0000ffff / (double)(nBits & 0x00ffffff);
    while (nShift < 29) {
        dDiff *= 256.0;
        nShift++;
    }
    while (nShift > 29) {
        dDiff /= 256.0;
        nShift--;
    }
    return dDiff;
}

} // namespace bcp
