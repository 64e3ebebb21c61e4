// Control/util RPCs. Parity: reference src/rpc/misc.cpp (table :586: getinfo,
// getmemoryinfo, validateaddress, createmultisig, verifymessage, signmessagewithprivkey,
// setmocktime, echo, echojson), src/rpc/server.cpp (help, stop, uptime) and
// src/rpc/abc.cpp (getexcessiveblock/setexcessiveblock, :77).
#include "keys/key.h"
#include "rpc/console.h"
#include "node/node.h"
#include "node/policy.h"
#include "node/sigverify.h"
#include "node/txmempool.h"
#include "rpc/core_io.h"
#include "net/net.h"
#include "rpc/server.h"
#include "script/sign.h"
#include "script/standard.h"
#include "kernels/gpu_api.h"
#include "node/gpuverify.h"
#include "node/miner.h"
#include "util/lockedpool.h"
#include "util/strencodings.h"

#include <mutex>

namespace bcp {

static NodeContext& Node() {
    NodeContext* n = GetNode();
    if (!n || !n->chainstate) ThrowRPC(RPC_INTERNAL_ERROR, "node not initialised");
    return *n;
}
double GetDifficulty(const CBlockIndex* blockindex);

// Wallet hooks (filled in by the wallet module when enabled).
std::function<CScript()> g_walletMiningScript;
std::function<void(UniValue&)> g_walletGetInfo;
std::function<bool(const CTxDestination&, UniValue&)> g_walletDescribeAddress;

CScript GetScriptForMining() {
    if (g_walletMiningScript) return g_walletMiningScript();
    // no wallet: pay to a node-local key (kept in memory for the process lifetime)
    static std::once_flag once;
    static CKey key;
    std::call_once(once, [] { key.MakeNewKey(true); });
    return GetScriptForRawPubKey(key.GetPubKey());
}

static UniValue help(const JSONRPCRequest& req) {
    std::string strCommand;
    if (req.params.size() > 0) strCommand = req.params[0].get_str();
    return tableRPC.help(strCommand);
}

static UniValue stop(const JSONRPCRequest& req) {
    RequestShutdown();
    return "Bitcoin Cash Plus server stopping";
}

static UniValue uptime(const JSONRPCRequest& req) { return GetTime() - GetStartupTime(); }

static UniValue getinfo(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("version", CLIENT_VERSION);
    obj.pushKV("protocolversion", PROTOCOL_VERSION);
    if (g_walletGetInfo) g_walletGetInfo(obj);
    obj.pushKV("blocks", cs.Height());
    obj.pushKV("timeoffset", GetTimeOffset());
    obj.pushKV("connections", GetConnman() ? (int64_t)GetConnman()->GetNodeCount(CONNECTIONS_ALL) : (int64_t)0);
    obj.pushKV("proxy", "");
    obj.pushKV("difficulty", GetDifficulty(cs.Tip()));
    obj.pushKV("testnet", cs.Params().NetworkIDString() == "test");
    obj.pushKV("paytxfee", ValueFromAmount(0));
    obj.pushKV("relayfee", ValueFromAmount(minRelayTxFee.GetFeePerK()));
    obj.pushKV("errors", cs.Warnings());
    return obj;
}

static UniValue getmemoryinfo(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    UniValue obj(UniValue::VOBJ);
    UniValue locked(UniValue::VOBJ);
    const LockedPool::Stats st = LockedPoolManager::Instance().stats();
    locked.pushKV("used", (int64_t)st.used);
    locked.pushKV("free", (int64_t)st.free);
    locked.pushKV("total", (int64_t)st.total);
    locked.pushKV("locked", (int64_t)st.locked);
    locked.pushKV("chunks_used", (int64_t)st.chunks_used);
    locked.pushKV("chunks_free", (int64_t)st.chunks_free);
    obj.pushKV("locked", locked);
    obj.pushKV("coins_cache_bytes", (int64_t)n.chainstate->CoinsTip().DynamicMemoryUsage());
    obj.pushKV("mempool_bytes", (int64_t)n.mempool->DynamicMemoryUsage());
    obj.pushKV("sigcache_entries", (int64_t)GetSignatureCache().Size());
    return obj;
}

// GPU accelerator status (MI355X): device, kernels used by validation and mining.
static UniValue getgpuinfo(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    UniValue obj(UniValue::VOBJ);
    const bool avail = gpu::GpuAvailable();
    obj.pushKV("available", avail);
    obj.pushKV("enabled", n.useGpu);
    if (avail) {
        obj.pushKV("devices", gpu::DeviceCount());
        obj.pushKV("name", gpu::DeviceName(0));
    }
    const SigVerifyStats s = GetSigVerifyStats();
    UniValue sv(UniValue::VOBJ);
    sv.pushKV("gpu_batches", (uint64_t)s.gpu_batches);
    sv.pushKV("gpu_sigs", (uint64_t)s.gpu_sigs);
    sv.pushKV("cpu_sigs", (uint64_t)s.cpu_sigs);
    sv.pushKV("cache_hits", (uint64_t)s.cache_hits);
    sv.pushKV("multisig_groups", (uint64_t)s.multisig_groups);
    sv.pushKV("gpu_ms", s.gpu_ms);
    sv.pushKV("cpu_ms", s.cpu_ms);
    sv.pushKV("gpu_threshold", (uint64_t)GetGpuSigThreshold());
    sv.pushKV("gpu_failures", (uint64_t)s.gpu_failures);
    sv.pushKV("gpu_disabled", GpuSigPathDisabled());
    obj.pushKV("sigverify", sv);
    // validation lanes (node/gpuverify.h): devices, stream priority, work done per lane
    GpuVerifyService& svc = GpuVerifyService::Instance();
    UniValue vd(UniValue::VARR);
    for (int d : svc.Devices()) vd.push_back(d);
    obj.pushKV("validation_devices", vd);
    UniValue lanes(UniValue::VARR);
    for (const auto& L : svc.Stats()) {
        UniValue o(UniValue::VOBJ);
        o.pushKV("device", L.device);
        o.pushKV("stream_priority", L.priority);
        o.pushKV("batches", L.batches);
        o.pushKV("items", L.items);
        o.pushKV("ecdsa_items", L.ecdsaItems);
        o.pushKV("equihash_items", L.equihashItems);
        lanes.push_back(o);
    }
    obj.pushKV("validation_lanes", lanes);
    obj.pushKV("sharded_batches", svc.ShardedBatches());
    UniValue md(UniValue::VARR);
    if (avail)
        for (int d : GetMinerGpuDevices()) md.push_back(d);
    obj.pushKV("miner_devices", md);
    return obj;
}

static UniValue setgpusigthreshold(const JSONRPCRequest& req) {
    SetGpuSigThreshold((size_t)req.params[0].get_int64());
    return UniValue::NullUniValue;
}

static UniValue validateaddress(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "validateaddress \"address\"");
    const CChainParams& params = Node().chainstate->Params();
    CTxDestination dest = DecodeDestination(req.params[0].get_str(), params);
    const bool isValid = dest.IsValid();
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("isvalid", isValid);
    if (isValid) {
        const std::string currentAddress = EncodeDestination(dest, params);
        ret.pushKV("address", currentAddress);
        CScript scriptPubKey = GetScriptForDestination(dest);
        ret.pushKV("scriptPubKey", HexStr(scriptPubKey.begin(), scriptPubKey.end()));
        ret.pushKV("isscript", dest.type == DestType::SCRIPTID);
        if (g_walletDescribeAddress) g_walletDescribeAddress(dest, ret);
        else {
            ret.pushKV("ismine", false);
            ret.pushKV("iswatchonly", false);
        }
    }
    return ret;
}

// Parse a pubkey (hex) or, with a wallet, an address whose key is known.
CScript CreateMultisigRedeemscript(const UniValue& params) {
    const int nRequired = params[0].get_int();
    const UniValue& keys = params[1].get_array();
    if (nRequired < 1) ThrowRPC(RPC_INVALID_PARAMETER, "a multisignature address must require at least one key to redeem");
    if ((int)keys.size() < nRequired)
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("not enough keys supplied (got %u keys, but need at least %d to redeem)",
                                                  (unsigned)keys.size(), nRequired));
    if (keys.size() > 16) ThrowRPC(RPC_INVALID_PARAMETER, "Number of addresses involved in the multisignature address creation > 16\nReduce the number");
    NodeContext& n = Node();
    std::vector<CPubKey> pubkeys;
    for (size_t i = 0; i < keys.size(); i++) {
        const std::string& ks = keys[i].get_str();
        CTxDestination dest = DecodeDestination(ks, n.chainstate->Params());
        if (n.keystore && dest.IsValid() && dest.type == DestType::KEYID) {
            CPubKey vchPubKey;
            if (!n.keystore->GetPubKey(CKeyID(dest.hash), vchPubKey))
                ThrowRPC(RPC_INVALID_PARAMETER, strprintf("no full public key for address %s", ks.c_str()));
            if (!vchPubKey.IsFullyValid()) ThrowRPC(RPC_INVALID_PARAMETER, " Invalid public key: " + ks);
            pubkeys.push_back(vchPubKey);
        } else if (IsHex(ks)) {
            CPubKey vchPubKey(ParseHex(ks));
            if (!vchPubKey.IsFullyValid()) ThrowRPC(RPC_INVALID_PARAMETER, " Invalid public key: " + ks);
            pubkeys.push_back(vchPubKey);
        } else {
            ThrowRPC(RPC_INVALID_PARAMETER, " Invalid public key: " + ks);
        }
    }
    CScript result = GetScriptForMultisig(nRequired, pubkeys);
    if (result.size() > MAX_SCRIPT_ELEMENT_SIZE)
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("redeemScript exceeds size limit: %u > %u", (unsigned)result.size(),
                                                  MAX_SCRIPT_ELEMENT_SIZE));
    return result;
}

static UniValue createmultisig(const JSONRPCRequest& req) {
    if (req.params.size() != 2) ThrowRPC(RPC_INVALID_PARAMS, "createmultisig nrequired [\"key\",...]");
    CScript inner = CreateMultisigRedeemscript(req.params);
    CScriptID innerID(inner);
    UniValue result(UniValue::VOBJ);
    result.pushKV("address", EncodeDestination(CTxDestination(innerID), Node().chainstate->Params()));
    result.pushKV("redeemScript", HexStr(inner.begin(), inner.end()));
    return result;
}

static UniValue verifymessage(const JSONRPCRequest& req) {
    if (req.params.size() != 3) ThrowRPC(RPC_INVALID_PARAMS, "verifymessage \"address\" \"signature\" \"message\"");
    const std::string strAddress = req.params[0].get_str();
    const std::string strSign = req.params[1].get_str();
    const std::string strMessage = req.params[2].get_str();
    CTxDestination dest = DecodeDestination(strAddress, Node().chainstate->Params());
    if (!dest.IsValid()) ThrowRPC(RPC_TYPE_ERROR, "Invalid address");
    if (dest.type != DestType::KEYID) ThrowRPC(RPC_TYPE_ERROR, "Address does not refer to key");
    bool fInvalid = false;
    std::vector<unsigned char> vchSig = DecodeBase64(strSign, &fInvalid);
    if (fInvalid) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Malformed base64 encoding");
    CPubKey pubkey;
    if (!pubkey.RecoverCompact(MessageHash(strMessage), vchSig)) return false;
    return pubkey.GetID() == CKeyID(dest.hash);
}

static UniValue signmessagewithprivkey(const JSONRPCRequest& req) {
    if (req.params.size() != 2) ThrowRPC(RPC_INVALID_PARAMS, "signmessagewithprivkey \"privkey\" \"message\"");
    CKey key = DecodeSecret(req.params[0].get_str(), Node().chainstate->Params());
    if (!key.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid private key");
    std::vector<unsigned char> vchSig;
    if (!key.SignCompact(MessageHash(req.params[1].get_str()), vchSig)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Sign failed");
    return EncodeBase64(vchSig.data(), vchSig.size());
}

static UniValue setmocktime(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "setmocktime timestamp");
    if (!Node().chainstate->Params().MineBlocksOnDemand()) ThrowRPC(RPC_METHOD_NOT_FOUND, "setmocktime for regression testing (-regtest mode) only");
    SetMockTime(req.params[0].get_int64());
    return UniValue::NullUniValue;
}

static UniValue echo(const JSONRPCRequest& req) { return req.params; }

// ---- abc.cpp: excessive block size
static UniValue getexcessiveblock(const JSONRPCRequest& req) {
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("excessiveBlockSize", (uint64_t)Node().chainstate->MaxBlockSize());
    return ret;
}
static UniValue setexcessiveblock(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "setexcessiveblock blockSize");
    uint64_t ebs = 0;
    if (req.params[0].isNum()) ebs = (uint64_t)req.params[0].get_int64();
    else {
        const std::string temp = req.params[0].get_str();
        if (temp[0] == '-') throw std::runtime_error("setexcessiveblock blockSize");
        ebs = (uint64_t)atoi64(temp);
    }
    if (!Node().chainstate->SetMaxBlockSize(ebs))
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("Invalid parameter, excessiveblock must be larger than %llu",
                                                  (unsigned long long)LEGACY_MAX_BLOCK_SIZE));
    return "Excessive Block set to " + std::to_string(ebs) + " bytes.";
}

// Console line execution for the browser GUI console (reference Qt RPCConsole::RPCExecuteCommandLine):
// nested calls, [key] result queries, and the history-filtered form of the line.
static UniValue execconsole(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "execconsole \"line\"");
    const std::string line = req.params[0].get_str();
    UniValue r(UniValue::VOBJ);
    std::string filtered, result;
    // the history form is computed without executing, so it exists even when execution fails
    try {
        std::string dummy;
        RPCParseCommandLine(dummy, line, nullptr, &filtered);
    } catch (const std::exception&) {
        filtered = IsSensitiveConsoleCommand(line.substr(0, line.find_first_of(" (\t"))) ? "" : line;
    }
    const ConsoleExecutor exec = [](const std::string& m, const std::vector<std::string>& a) {
        if (m == "execconsole") ThrowRPC(RPC_INVALID_PARAMETER, "execconsole cannot be nested");
        return ConsoleExecuteRPC(m, a);
    };
    try {
        RPCParseCommandLine(result, line, &exec);
    } catch (const std::runtime_error& e) {
        ThrowRPC(RPC_PARSE_ERROR, e.what());
    }
    r.pushKV("result", result);
    r.pushKV("filtered", filtered);
    return r;
}

void RegisterMiscRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"hidden", "execconsole", execconsole, true, {"line"}, "execconsole \"line\"\nRun one RPC console line (nested calls such as getblock(getbestblockhash())[tx][0]); returns the result and the history-filtered line."},
        {"control", "help", help, true, {"command"}, "help ( \"command\" )\nList all commands, or get help for a specified command."},
        {"control", "stop", stop, true, {}, "stop\nStop Bitcoin Cash Plus server."},
        {"control", "uptime", uptime, true, {}, "uptime\nReturns the total uptime of the server."},
        {"control", "getinfo", getinfo, true, {}, "getinfo\nDEPRECATED. Returns an object containing various state info."},
        {"control", "getmemoryinfo", getmemoryinfo, true, {}, "getmemoryinfo\nReturns an object containing information about memory usage."},
        {"control", "getgpuinfo", getgpuinfo, true, {}, "getgpuinfo\nReturns MI355X accelerator status and batched-verification statistics."},
        {"hidden", "setgpusigthreshold", setgpusigthreshold, true, {"n"}, "setgpusigthreshold n\nMinimum ECDSA batch size routed to the GPU."},
        {"util", "validateaddress", validateaddress, true, {"address"}, "validateaddress \"address\"\nReturn information about the given bitcoin address."},
        {"util", "createmultisig", createmultisig, true, {"nrequired", "keys"}, "createmultisig nrequired [\"key\",...]\nCreates a multi-signature address with n signature of m keys required."},
        {"util", "verifymessage", verifymessage, true, {"address", "signature", "message"}, "verifymessage \"address\" \"signature\" \"message\"\nVerify a signed message."},
        {"util", "signmessagewithprivkey", signmessagewithprivkey, true, {"privkey", "message"}, "signmessagewithprivkey \"privkey\" \"message\"\nSign a message with the private key of an address."},
        {"hidden", "setmocktime", setmocktime, true, {"timestamp"}, "setmocktime timestamp\nSet the local time to given timestamp (-regtest only)."},
        {"hidden", "echo", echo, true, {"arg0", "arg1", "arg2", "arg3", "arg4", "arg5", "arg6", "arg7", "arg8", "arg9"}, "echo|echojson \"message\" ...\nSimply echo back the input arguments."},
        {"hidden", "echojson", echo, true, {"arg0", "arg1", "arg2", "arg3", "arg4", "arg5", "arg6", "arg7", "arg8", "arg9"}, "echojson ...\nSimply echo back the input arguments."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

void RegisterABCRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"network", "getexcessiveblock", getexcessiveblock, true, {}, "getexcessiveblock\nReturn the excessive block size."},
        {"network", "setexcessiveblock", setexcessiveblock, true, {"maxBlockSize"}, "setexcessiveblock blockSize\nSet the excessive block size. Excessive blocks will not be used in the active chain or relayed."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
