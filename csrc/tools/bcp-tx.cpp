// bcp-tx: offline transaction builder / editor / signer.
// Parity: reference src/bitcoin-tx.cpp (commands delin, delout, in, locktime, nversion,
// outaddr, outdata, outmultisig, outpubkey, outscript, sign, load, set; -create, -json,
// -txid, chain selection; legacy-address JSON output) and its golden test suite
// src/test/data/bitcoin-util-test.json (run by tests/test_bcp_tx.py).
#include "consensus/params.h"
#include "consensus/tx_verify.h"
#include "keys/key.h"
#include "primitives/transaction.h"
#include "rpc/core_io.h"
#include "rpc/server.h"
#include "script/sign.h"
#include "script/standard.h"
#include "util/strencodings.h"
#include "util/univalue.h"
#include "util/util.h"

#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

using namespace bcp;

static std::map<std::string, UniValue> registers;

static std::vector<std::string> Split(const std::string& s, char sep) {
    std::vector<std::string> out;
    size_t start = 0;
    for (;;) {
        const size_t p = s.find(sep, start);
        out.push_back(s.substr(start, p == std::string::npos ? std::string::npos : p - start));
        if (p == std::string::npos) break;
        start = p + 1;
    }
    return out;
}

static Amount ExtractAndValidateValue(const std::string& s) {
    int64_t v;
    if (!ParseMoney(s, v)) throw std::runtime_error("invalid TX output value");
    return v;
}

static void RegisterSetJson(const std::string& key, const std::string& rawJson) {
    UniValue val;
    if (!val.read(rawJson)) throw std::runtime_error("Cannot parse JSON for key " + key);
    registers[key] = val;
}

static void RegisterSet(const std::string& strInput) {
    const size_t pos = strInput.find(':');
    if (pos == std::string::npos || pos == 0 || pos == strInput.size() - 1)
        throw std::runtime_error("Register input requires NAME:VALUE");
    RegisterSetJson(strInput.substr(0, pos), strInput.substr(pos + 1));
}

static void RegisterLoad(const std::string& strInput) {
    const size_t pos = strInput.find(':');
    if (pos == std::string::npos || pos == 0 || pos == strInput.size() - 1)
        throw std::runtime_error("Register load requires NAME:FILENAME");
    const std::string key = strInput.substr(0, pos), filename = strInput.substr(pos + 1);
    std::ifstream f(filename);
    if (!f) throw std::runtime_error("Cannot open file " + filename);
    std::stringstream ss;
    ss << f.rdbuf();
    RegisterSetJson(key, ss.str());
}

static void MutateTxVersion(CMutableTransaction& tx, const std::string& s) {
    const int64_t v = atoi64(s);
    if (v < 1 || v > CTransaction::MAX_STANDARD_VERSION) throw std::runtime_error("Invalid TX version requested");
    tx.nVersion = (int)v;
}

static void MutateTxLocktime(CMutableTransaction& tx, const std::string& s) {
    const int64_t v = atoi64(s);
    if (v < 0 || v > 0xffffffffLL) throw std::runtime_error("Invalid TX locktime requested");
    tx.nLockTime = (uint32_t)v;
}

static void MutateTxAddInput(CMutableTransaction& tx, const std::string& s) {
    const std::vector<std::string> v = Split(s, ':');
    if (v.size() < 2 || v.size() > 3) throw std::runtime_error("TX input missing separator");
    if (v[0].size() != 64 || !IsHex(v[0])) throw std::runtime_error("invalid TX input txid");
    const uint256 txid = uint256S(v[0]);
    static const unsigned int minTxOutSz = 9;
    static const unsigned int maxVout = MAX_TX_SIZE / minTxOutSz;
    const int vout = atoi(v[1].c_str());
    if (vout < 0 || (unsigned)vout > maxVout) throw std::runtime_error("invalid TX input vout");
    uint32_t nSequence = CTxIn::SEQUENCE_FINAL;
    if (v.size() > 2) nSequence = (uint32_t)atoi64(v[2]);
    tx.vin.push_back(CTxIn(COutPoint(txid, (uint32_t)vout), CScript(), nSequence));
}

static void MutateTxAddOutAddr(CMutableTransaction& tx, const std::string& s) {
    const std::vector<std::string> v = Split(s, ':');
    if (v.size() != 2) throw std::runtime_error("TX output missing or too many separators");
    const Amount value = ExtractAndValidateValue(v[0]);
    const CTxDestination d = DecodeDestination(v[1], Params());
    if (!d.IsValid()) throw std::runtime_error("invalid TX output address");
    tx.vout.push_back(CTxOut(value, GetScriptForDestination(d)));
}

static void MutateTxAddOutPubKey(CMutableTransaction& tx, const std::string& s) {
    const std::vector<std::string> v = Split(s, ':');
    if (v.size() < 2 || v.size() > 3) throw std::runtime_error("TX output missing or too many separators");
    const Amount value = ExtractAndValidateValue(v[0]);
    const std::vector<unsigned char> pk = ParseHex(v[1]);
    const CPubKey pub(pk.begin(), pk.end());
    if (!pub.IsFullyValid()) throw std::runtime_error("invalid TX output pubkey");
    CScript spk = GetScriptForRawPubKey(pub);
    if (v.size() == 3) {
        if (v[2].find('S') != std::string::npos) spk = GetScriptForDestination(CScriptID(spk));
        else throw std::runtime_error("unknown output flags");
    }
    tx.vout.push_back(CTxOut(value, spk));
}

static void MutateTxAddOutMultiSig(CMutableTransaction& tx, const std::string& s) {
    const std::vector<std::string> v = Split(s, ':');
    if (v.size() < 3) throw std::runtime_error("Not enough multisig parameters");
    const Amount value = ExtractAndValidateValue(v[0]);
    const uint32_t required = (uint32_t)atoi(v[1].c_str());
    const uint32_t numkeys = (uint32_t)atoi(v[2].c_str());
    if (v.size() < numkeys + 3 || v.size() > numkeys + 4) throw std::runtime_error("incorrect number of multisig pubkeys");
    if (required < 1 || required > 20 || numkeys < 1 || numkeys > 20 || numkeys < required)
        throw std::runtime_error("multisig parameter mismatch. Required " + std::to_string(required) + " of " +
                                 std::to_string(numkeys) + "signatures.");
    std::vector<CPubKey> pubkeys;
    for (uint32_t i = 0; i < numkeys; i++) {
        const std::vector<unsigned char> pk = ParseHex(v[3 + i]);
        const CPubKey pub(pk.begin(), pk.end());
        if (!pub.IsFullyValid()) throw std::runtime_error("invalid TX output pubkey");
        pubkeys.push_back(pub);
    }
    CScript spk = GetScriptForMultisig((int)required, pubkeys);
    if (v.size() == numkeys + 4) {
        if (v.back().find('S') != std::string::npos) spk = GetScriptForDestination(CScriptID(spk));
        else throw std::runtime_error("unknown output flags");
    }
    tx.vout.push_back(CTxOut(value, spk));
}

static void MutateTxAddOutData(CMutableTransaction& tx, const std::string& s) {
    Amount value = 0;
    const size_t pos = s.find(':');
    if (pos == 0) throw std::runtime_error("TX output value not specified");
    if (pos != std::string::npos) value = ExtractAndValidateValue(s.substr(0, pos));
    const std::string hex = s.substr(pos == std::string::npos ? 0 : pos + 1);
    if (!IsHex(hex)) throw std::runtime_error("invalid TX output data");
    const std::vector<unsigned char> data = ParseHex(hex);
    CScript spk;
    spk << OP_RETURN << data;
    tx.vout.push_back(CTxOut(value, spk));
}

static void MutateTxAddOutScript(CMutableTransaction& tx, const std::string& s) {
    const std::vector<std::string> v = Split(s, ':');
    if (v.size() < 2 || v.size() > 3) throw std::runtime_error("TX output missing separator");
    const Amount value = ExtractAndValidateValue(v[0]);
    CScript spk = ParseScript(v[1]);
    if (v.size() == 3) {
        if (v[2].find('S') != std::string::npos) spk = GetScriptForDestination(CScriptID(spk));
        else throw std::runtime_error("unknown output flags");
    }
    tx.vout.push_back(CTxOut(value, spk));
}

static void MutateTxDelInput(CMutableTransaction& tx, const std::string& s) {
    const int idx = atoi(s.c_str());
    if (idx < 0 || idx >= (int)tx.vin.size()) throw std::runtime_error("Invalid TX input index '" + s + "'");
    tx.vin.erase(tx.vin.begin() + idx);
}

static void MutateTxDelOutput(CMutableTransaction& tx, const std::string& s) {
    const int idx = atoi(s.c_str());
    if (idx < 0 || idx >= (int)tx.vout.size()) throw std::runtime_error("Invalid TX output index '" + s + "'");
    tx.vout.erase(tx.vout.begin() + idx);
}

static const std::pair<const char*, uint32_t> kSighashOptions[] = {
    {"ALL", SIGHASH_ALL},
    {"NONE", SIGHASH_NONE},
    {"SINGLE", SIGHASH_SINGLE},
    {"ALL|ANYONECANPAY", SIGHASH_ALL | SIGHASH_ANYONECANPAY},
    {"NONE|ANYONECANPAY", SIGHASH_NONE | SIGHASH_ANYONECANPAY},
    {"SINGLE|ANYONECANPAY", SIGHASH_SINGLE | SIGHASH_ANYONECANPAY},
    {"ALL|FORKID", SIGHASH_ALL | SIGHASH_FORKID},
    {"NONE|FORKID", SIGHASH_NONE | SIGHASH_FORKID},
    {"SINGLE|FORKID", SIGHASH_SINGLE | SIGHASH_FORKID},
    {"ALL|FORKID|ANYONECANPAY", SIGHASH_ALL | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
    {"NONE|FORKID|ANYONECANPAY", SIGHASH_NONE | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
    {"SINGLE|FORKID|ANYONECANPAY", SIGHASH_SINGLE | SIGHASH_FORKID | SIGHASH_ANYONECANPAY},
};

static void MutateTxSign(CMutableTransaction& tx, const std::string& flagStr) {
    uint32_t nHashType = SIGHASH_ALL | SIGHASH_FORKID;
    if (!flagStr.empty()) {
        bool found = false;
        for (const auto& o : kSighashOptions)
            if (flagStr == o.first) {
                nHashType = o.second;
                found = true;
            }
        if (!found) throw std::runtime_error("unknown sighash flag/sign option");
    }
    if (!registers.count("privatekeys")) throw std::runtime_error("privatekeys register variable must be set.");
    CBasicKeyStore keystore;
    const UniValue keys = registers["privatekeys"].get_array();
    for (size_t i = 0; i < keys.size(); i++) {
        if (!keys[i].isStr()) throw std::runtime_error("privatekey not a std::string");
        const CKey key = DecodeSecret(keys[i].get_str(), Params());
        if (!key.IsValid()) throw std::runtime_error("privatekey not valid");
        keystore.AddKey(key);
    }
    if (!registers.count("prevtxs")) throw std::runtime_error("prevtxs register variable must be set.");
    const UniValue prevtxs = registers["prevtxs"].get_array();
    std::map<COutPoint, std::pair<CScript, Amount>> coins;
    for (size_t i = 0; i < prevtxs.size(); i++) {
        const UniValue& p = prevtxs[i];
        if (!p.isObject()) throw std::runtime_error("expected prevtxs internal object");
        const UniValue& txidV = find_value(p, "txid");
        const UniValue& voutV = find_value(p, "vout");
        const UniValue& spkV = find_value(p, "scriptPubKey");
        if (!txidV.isStr() || !voutV.isNum() || !spkV.isStr()) throw std::runtime_error("prevtxs internal object typecheck fail");
        const uint256 txid = uint256S(txidV.get_str());
        const int nOut = voutV.get_int();
        if (nOut < 0) throw std::runtime_error("vout must be positive");
        const std::vector<unsigned char> spkData = ParseHex(spkV.get_str());
        const CScript spk(spkData.begin(), spkData.end());
        Amount amount = 0;
        const UniValue& amt = find_value(p, "amount");
        if (!amt.isNull()) amount = AmountFromValue(amt);
        coins[COutPoint(txid, (uint32_t)nOut)] = {spk, amount};
        // P2SH redeem scripts
        const UniValue& rs = find_value(p, "redeemScript");
        if (spk.IsPayToScriptHash() && rs.isStr()) {
            const std::vector<unsigned char> rd = ParseHex(rs.get_str());
            keystore.AddCScript(CScript(rd.begin(), rd.end()));
        }
    }
    const bool fHashSingle = (nHashType & ~(SIGHASH_ANYONECANPAY | SIGHASH_FORKID)) == SIGHASH_SINGLE;
    const CMutableTransaction mergedBase = tx;
    for (unsigned i = 0; i < tx.vin.size(); i++) {
        auto it = coins.find(tx.vin[i].prevout);
        if (it == coins.end()) continue;
        const CScript& prevPubKey = it->second.first;
        const Amount amount = it->second.second;
        SignatureData sigdata;
        if (!fHashSingle || i < tx.vout.size()) {
            const CTransaction txConst(mergedBase);
            ProduceSignature(TransactionSignatureCreator(&keystore, &txConst, i, amount, nHashType), prevPubKey, sigdata);
        }
        sigdata = CombineSignatures(prevPubKey, MutableTransactionSignatureChecker(&tx, i, amount), sigdata,
                                    DataFromTransaction(tx, i));
        UpdateTransaction(tx, i, sigdata);
    }
}

static void MutateTx(CMutableTransaction& tx, const std::string& command, const std::string& value) {
    if (command == "nversion") MutateTxVersion(tx, value);
    else if (command == "locktime") MutateTxLocktime(tx, value);
    else if (command == "delin") MutateTxDelInput(tx, value);
    else if (command == "in") MutateTxAddInput(tx, value);
    else if (command == "delout") MutateTxDelOutput(tx, value);
    else if (command == "outaddr") MutateTxAddOutAddr(tx, value);
    else if (command == "outpubkey") MutateTxAddOutPubKey(tx, value);
    else if (command == "outmultisig") MutateTxAddOutMultiSig(tx, value);
    else if (command == "outdata") MutateTxAddOutData(tx, value);
    else if (command == "outscript") MutateTxAddOutScript(tx, value);
    else if (command == "sign") MutateTxSign(tx, value);
    else if (command == "load") RegisterLoad(value);
    else if (command == "set") RegisterSet(value);
    else throw std::runtime_error("unknown command");
}

static void Usage() {
    printf("%s bcp-tx utility version %s\n\n", CLIENT_NAME, FormatFullVersion().c_str());
    printf("Usage:  bcp-tx [options] <hex-tx> [commands]  Update hex-encoded transaction\n"
           "or:     bcp-tx [options] -create [commands]   Create hex-encoded transaction\n\n"
           "Options:\n  -create  Create new, empty TX.\n  -json  Select JSON output\n"
           "  -txid  Output only the hex-encoded transaction id of the resultant transaction.\n"
           "  -testnet / -regtest  Chain selection\n\nCommands:\n"
           "  delin=N  delout=N  in=TXID:VOUT(:SEQUENCE_NUMBER)  locktime=N  nversion=N\n"
           "  outaddr=VALUE:ADDRESS  outdata=[VALUE:]DATA  outpubkey=VALUE:PUBKEY[:FLAGS]\n"
           "  outmultisig=VALUE:REQUIRED:PUBKEYS:PUBKEY1:PUBKEY2:....[:FLAGS]  outscript=VALUE:SCRIPT[:FLAGS]\n"
           "  sign=SIGHASH-FLAGS (requires privatekeys and prevtxs registers)\n"
           "  load=NAME:FILENAME  set=NAME:JSON-STRING\n");
}

int main(int argc, char* argv[]) {
    int first = 1;
    while (first < argc && argv[first][0] == '-' && argv[first][1] != '\0' && !(argv[first][1] >= '0' && argv[first][1] <= '9'))
        first++;
    gArgs.ParseParameters(first, argv);
    if (gArgs.IsArgSet("-?") || gArgs.IsArgSet("-h") || gArgs.IsArgSet("-help")) {
        Usage();
        return argc < 2 ? 1 : 0;
    }
    try {
        SelectParams(gArgs.GetChainName());
    } catch (const std::exception& e) {
        fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    SetUseCashAddr(gArgs.GetBoolArg("-usecashaddr", false));
    std::vector<std::string> args(argv + first, argv + argc);
    const bool fCreateBlank = gArgs.GetBoolArg("-create", false);
    try {
        CMutableTransaction tx;
        size_t start = 0;
        if (!fCreateBlank) {
            if (args.empty()) throw std::runtime_error("too few parameters");
            std::string hex = args[0];
            if (hex == "-") {
                std::stringstream ss;
                ss << std::cin.rdbuf();
                hex = TrimString(ss.str());
            }
            if (!DecodeHexTx(tx, hex)) throw std::runtime_error("invalid transaction encoding");
            start = 1;
        }
        for (size_t i = start; i < args.size(); i++) {
            const std::string& a = args[i];
            const size_t eq = a.find('=');
            if (eq == std::string::npos) throw std::runtime_error("unknown command");
            MutateTx(tx, a.substr(0, eq), a.substr(eq + 1));
        }
        const CTransaction out(tx);
        if (gArgs.GetBoolArg("-json", false)) {
            UniValue entry(UniValue::VOBJ);
            TxToUniv(out, uint256(), entry, Params(), false);
            printf("%s\n", entry.write(4).c_str());
        } else if (gArgs.GetBoolArg("-txid", false)) {
            printf("%s\n", out.GetHash().GetHex().c_str());
        } else {
            printf("%s\n", EncodeHexTx(out).c_str());
        }
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
