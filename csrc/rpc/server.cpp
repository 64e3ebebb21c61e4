#include "rpc/server.h"
#include "node/warnings.h"
#include "keys/key.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <atomic>
#include <cmath>
#include <fstream>

namespace bcp {

CRPCTable tableRPC;

UniValue JSONRPCError(int code, const std::string& message) {
    UniValue error(UniValue::VOBJ);
    error.pushKV("code", code);
    error.pushKV("message", message);
    return error;
}
void ThrowRPC(int code, const std::string& message) { throw JSONRPCException{JSONRPCError(code, message)}; }

UniValue JSONRPCRequestObj(const std::string& method, const UniValue& params, const UniValue& id) {
    UniValue r(UniValue::VOBJ);
    r.pushKV("method", method);
    r.pushKV("params", params);
    r.pushKV("id", id);
    return r;
}
UniValue JSONRPCReplyObj(const UniValue& result, const UniValue& error, const UniValue& id) {
    UniValue reply(UniValue::VOBJ);
    if (!error.isNull()) reply.pushKV("result", UniValue::NullUniValue);
    else reply.pushKV("result", result);
    reply.pushKV("error", error);
    reply.pushKV("id", id);
    return reply;
}

void JSONRPCRequest::parse(const UniValue& valRequest) {
    if (!valRequest.isObject()) ThrowRPC(RPC_INVALID_REQUEST, "Invalid Request object");
    const UniValue& request = valRequest.get_obj();
    id = request["id"];
    const UniValue& valMethod = request["method"];
    if (valMethod.isNull()) ThrowRPC(RPC_INVALID_REQUEST, "Missing method");
    if (!valMethod.isStr()) ThrowRPC(RPC_INVALID_REQUEST, "Method must be a string");
    strMethod = valMethod.get_str();
    const UniValue& valParams = request["params"];
    if (valParams.isArray() || valParams.isObject()) params = valParams;
    else if (valParams.isNull()) params = UniValue(UniValue::VARR);
    else ThrowRPC(RPC_INVALID_REQUEST, "Params must be an array or object");
}

bool CRPCTable::appendCommand(const std::string& name, const CRPCCommand& cmd) {
    if (mapCommands.count(name)) return false;
    mapCommands[name] = cmd;
    return true;
}
const CRPCCommand* CRPCTable::operator[](const std::string& name) const {
    auto it = mapCommands.find(name);
    return it == mapCommands.end() ? nullptr : &it->second;
}
std::vector<std::string> CRPCTable::listCommands() const {
    std::vector<std::string> r;
    for (const auto& kv : mapCommands) r.push_back(kv.first);
    return r;
}

std::string CRPCTable::help(const std::string& strCommand) const {
    std::string strRet, category;
    std::vector<const CRPCCommand*> cmds;
    for (const auto& kv : mapCommands) cmds.push_back(&kv.second);
    std::sort(cmds.begin(), cmds.end(), [](const CRPCCommand* a, const CRPCCommand* b) {
        return a->category != b->category ? a->category < b->category : a->name < b->name;
    });
    for (const CRPCCommand* c : cmds) {
        if (!strCommand.empty() && c->name != strCommand) continue;
        if (c->category == "hidden" && strCommand.empty()) continue;
        if (!strCommand.empty()) return c->help.empty() ? c->name : c->help;
        if (c->category != category) {
            if (!category.empty()) strRet += "\n";
            category = c->category;
            std::string cat = category;
            if (!cat.empty()) cat[0] = (char)toupper(cat[0]);
            strRet += "== " + cat + " ==\n";
        }
        const std::string first = c->help.substr(0, c->help.find('\n'));
        strRet += (first.empty() ? c->name : first) + "\n";
    }
    if (strRet.empty()) strRet = strprintf("help: unknown command: %s\n", strCommand.c_str());
    if (!strRet.empty() && strRet.back() == '\n') strRet.pop_back();
    return strRet;
}

// Named parameters map onto positions by the command's argNames.
static JSONRPCRequest transformNamedArguments(const JSONRPCRequest& in, const std::vector<std::string>& argNames) {
    JSONRPCRequest out = in;
    out.params = UniValue(UniValue::VARR);
    const std::vector<std::string>& keys = in.params.getKeys();
    const std::vector<UniValue>& values = in.params.getValues();
    std::map<std::string, const UniValue*> argsIn;
    for (size_t i = 0; i < keys.size(); ++i) argsIn[keys[i]] = &values[i];
    int hole = 0;
    for (const std::string& argNamePattern : argNames) {
        // "a|b" alternatives
        std::vector<std::string> vargNames = SplitString(argNamePattern, '|');
        auto fr = argsIn.end();
        for (const std::string& n : vargNames) {
            fr = argsIn.find(n);
            if (fr != argsIn.end()) break;
        }
        if (fr != argsIn.end()) {
            for (int i = 0; i < hole; ++i) out.params.push_back(UniValue());
            hole = 0;
            out.params.push_back(*fr->second);
            argsIn.erase(fr);
        } else {
            hole += 1;
        }
    }
    if (!argsIn.empty()) ThrowRPC(RPC_INVALID_PARAMETER, "Unknown named parameter " + argsIn.begin()->first);
    return out;
}

UniValue CRPCTable::execute(const JSONRPCRequest& request) const {
    std::string status;
    if (RPCIsInWarmup(&status) && request.strMethod != "help" && request.strMethod != "stop")
        ThrowRPC(RPC_IN_WARMUP, status);
    const CRPCCommand* pcmd = (*this)[request.strMethod];
    if (!pcmd) ThrowRPC(RPC_METHOD_NOT_FOUND, "Method not found");
    if (!pcmd->okSafeMode) bcp::ObserveSafeMode();
    // more positional arguments than the command takes: its usage, as each reference handler
    // answers "if (request.fHelp || request.params.size() > N) throw runtime_error(help)"
    if (request.params.isArray() && request.params.size() > pcmd->argNames.size())
        ThrowRPC(RPC_MISC_ERROR, pcmd->help.empty() ? request.strMethod : pcmd->help);
    try {
        if (request.params.isObject()) return pcmd->actor(transformNamedArguments(request, pcmd->argNames));
        return pcmd->actor(request);
    } catch (const JSONRPCException&) {
        throw;
    } catch (const std::exception& e) {
        ThrowRPC(RPC_MISC_ERROR, e.what());
    }
}

static UniValue JSONRPCExecOne(const UniValue& req, const std::string& authUser) {
    JSONRPCRequest jreq;
    try {
        jreq.authUser = authUser;
        jreq.parse(req);
        UniValue result = tableRPC.execute(jreq);
        return JSONRPCReplyObj(result, UniValue::NullUniValue, jreq.id);
    } catch (const JSONRPCException& e) {
        return JSONRPCReplyObj(UniValue::NullUniValue, e.obj, jreq.id);
    } catch (const std::exception& e) {
        return JSONRPCReplyObj(UniValue::NullUniValue, JSONRPCError(RPC_PARSE_ERROR, e.what()), jreq.id);
    }
}

std::string JSONRPCExecute(const std::string& body, const std::string& authUser, int& httpStatus) {
    UniValue valRequest;
    httpStatus = 200;
    if (!valRequest.read(body)) {
        httpStatus = 500;
        return JSONRPCReplyObj(UniValue::NullUniValue, JSONRPCError(RPC_PARSE_ERROR, "Parse error"), UniValue()).write() + "\n";
    }
    if (valRequest.isObject()) {
        UniValue reply = JSONRPCExecOne(valRequest, authUser);
        // reference maps some errors to HTTP status codes (httprpc.cpp JSONErrorReply)
        const UniValue& err = reply["error"];
        if (!err.isNull()) {
            const int code = err["code"].isNum() ? err["code"].get_int() : 0;
            httpStatus = code == RPC_INVALID_REQUEST ? 400 : code == RPC_METHOD_NOT_FOUND ? 404 : 500;
        }
        return reply.write() + "\n";
    }
    if (valRequest.isArray()) {
        UniValue ret(UniValue::VARR);
        for (size_t i = 0; i < valRequest.size(); i++) ret.push_back(JSONRPCExecOne(valRequest[i], authUser));
        return ret.write() + "\n";
    }
    httpStatus = 500;
    return JSONRPCReplyObj(UniValue::NullUniValue, JSONRPCError(RPC_PARSE_ERROR, "Top-level object parse error"),
                           UniValue())
               .write() +
           "\n";
}

// ------------------------------------------------------------------ lifecycle
static std::mutex cs_warmup;
static bool fRPCInWarmup = true;
static std::string rpcWarmupStatus = "RPC server started";
static std::atomic<bool> fShutdown{false};
static std::function<void()> g_shutdownHook;
static const int64_t nStartupTime = GetTime();

void SetRPCWarmupStatus(const std::string& s) {
    std::lock_guard<std::mutex> l(cs_warmup);
    rpcWarmupStatus = s;
}
void SetRPCWarmupFinished() {
    std::lock_guard<std::mutex> l(cs_warmup);
    fRPCInWarmup = false;
}
bool RPCIsInWarmup(std::string* out) {
    std::lock_guard<std::mutex> l(cs_warmup);
    if (out) *out = rpcWarmupStatus;
    return fRPCInWarmup;
}
void SetRPCShutdownHook(std::function<void()> f) { g_shutdownHook = std::move(f); }
void RequestShutdown() {
    fShutdown = true;
    if (g_shutdownHook) g_shutdownHook();
}
bool ShutdownRequested() { return fShutdown.load(); }
int64_t GetStartupTime() { return nStartupTime; }

// ------------------------------------------------------------------ helpers
void RPCTypeCheckArgument(const UniValue& value, UniValue::VType typeExpected) {
    if (value.getType() != typeExpected)
        ThrowRPC(RPC_TYPE_ERROR, strprintf("Expected type %s, got %s", uvTypeName(typeExpected), uvTypeName(value.getType())));
}
void RPCTypeCheck(const UniValue& params, const std::vector<UniValue::VType>& types, bool fAllowNull) {
    for (size_t i = 0; i < types.size() && i < params.size(); i++) {
        const UniValue& v = params[i];
        if (!((v.getType() == types[i]) || (fAllowNull && v.isNull())))
            ThrowRPC(RPC_TYPE_ERROR, strprintf("Expected type %s, got %s", uvTypeName(types[i]), uvTypeName(v.getType())));
    }
}
uint256 ParseHashV(const UniValue& v, const std::string& strName) {
    std::string strHex;
    if (v.isStr()) strHex = v.get_str();
    if (!IsHex(strHex)) ThrowRPC(RPC_INVALID_PARAMETER, strName + " must be hexadecimal string (not '" + strHex + "')");
    if (strHex.size() != 64)
        ThrowRPC(RPC_INVALID_PARAMETER, strName + " must be of length 64 (not " + std::to_string(strHex.size()) + ")");
    return uint256S(strHex);
}
uint256 ParseHashO(const UniValue& o, const std::string& k) { return ParseHashV(o[k], k); }
std::vector<unsigned char> ParseHexV(const UniValue& v, const std::string& strName) {
    std::string strHex;
    if (v.isStr()) strHex = v.get_str();
    if (!IsHex(strHex)) ThrowRPC(RPC_INVALID_PARAMETER, strName + " must be hexadecimal string (not '" + strHex + "')");
    return ParseHex(strHex);
}
std::vector<unsigned char> ParseHexO(const UniValue& o, const std::string& k) { return ParseHexV(o[k], k); }

Amount AmountFromValue(const UniValue& value) {
    if (!value.isNum() && !value.isStr()) ThrowRPC(RPC_TYPE_ERROR, "Amount is not a number or string");
    int64_t amount;
    if (!ParseFixedPoint(value.getValStr(), 8, &amount)) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount");
    if (!MoneyRange(amount)) ThrowRPC(RPC_TYPE_ERROR, "Amount out of range");
    return amount;
}
UniValue ValueFromAmount(Amount amount) {
    const bool sign = amount < 0;
    const int64_t n_abs = sign ? -amount : amount;
    const int64_t quotient = n_abs / COIN;
    const int64_t remainder = n_abs % COIN;
    return UniValue(UniValue::VNUM, strprintf("%s%lld.%08lld", sign ? "-" : "", (long long)quotient, (long long)remainder));
}
std::string HelpExampleCli(const std::string& m, const std::string& a) { return "> bitcoincashplus-cli " + m + " " + a + "\n"; }
std::string HelpExampleRpc(const std::string& m, const std::string& a) {
    return "> curl --user myusername --data-binary '{\"jsonrpc\": \"1.0\", \"id\":\"curltest\", \"method\": \"" + m +
           "\", \"params\": [" + a + "] }' -H 'content-type: text/plain;' http://127.0.0.1:8332/\n";
}

// ------------------------------------------------------------------ CLI conversion
namespace {
struct ConvertParam {
    const char* method;
    int idx;
    const char* name;
};
const ConvertParam kConvert[] = {
    {"setmocktime", 0, "timestamp"}, {"generate", 0, "nblocks"}, {"generate", 1, "maxtries"},
    {"generatetoaddress", 0, "nblocks"}, {"generatetoaddress", 2, "maxtries"}, {"getnetworkhashps", 0, "nblocks"},
    {"getnetworkhashps", 1, "height"}, {"sendtoaddress", 1, "amount"}, {"sendtoaddress", 4, "subtractfeefromamount"},
    {"settxfee", 0, "amount"}, {"getreceivedbyaddress", 1, "minconf"}, {"getreceivedbyaccount", 1, "minconf"},
    {"listreceivedbyaddress", 0, "minconf"}, {"listreceivedbyaddress", 1, "include_empty"},
    {"listreceivedbyaddress", 2, "include_watchonly"}, {"listreceivedbyaccount", 0, "minconf"},
    {"listreceivedbyaccount", 1, "include_empty"}, {"listreceivedbyaccount", 2, "include_watchonly"},
    {"getbalance", 1, "minconf"}, {"getbalance", 2, "include_watchonly"}, {"getblockhash", 0, "height"},
    {"waitforblockheight", 0, "height"}, {"waitforblockheight", 1, "timeout"}, {"waitforblock", 1, "timeout"},
    {"waitfornewblock", 0, "timeout"}, {"move", 2, "amount"}, {"move", 3, "minconf"}, {"sendfrom", 2, "amount"},
    {"sendfrom", 3, "minconf"}, {"listtransactions", 1, "count"}, {"listtransactions", 2, "skip"},
    {"listtransactions", 3, "include_watchonly"}, {"listaccounts", 0, "minconf"}, {"listaccounts", 1, "include_watchonly"},
    {"walletpassphrase", 1, "timeout"}, {"getblocktemplate", 0, "template_request"},
    {"listsinceblock", 1, "target_confirmations"}, {"listsinceblock", 2, "include_watchonly"}, {"sendmany", 1, "amounts"}, {"sendwithcoincontrol", 0, "amounts"}, {"sendwithcoincontrol", 1, "inputs"}, {"sendwithcoincontrol", 3, "subtractfeefrom"},
    {"sendmany", 2, "minconf"}, {"sendmany", 4, "subtractfeefrom"}, {"addmultisigaddress", 0, "nrequired"},
    {"addmultisigaddress", 1, "keys"}, {"createmultisig", 0, "nrequired"}, {"createmultisig", 1, "keys"},
    {"listunspent", 0, "minconf"}, {"listunspent", 1, "maxconf"}, {"listunspent", 2, "addresses"},
    {"getblock", 1, "verbose"}, {"getblock", 2, "legacy"}, {"getblockheader", 1, "verbose"},
    {"gettransaction", 1, "include_watchonly"}, {"getrawtransaction", 1, "verbose"},
    {"createrawtransaction", 0, "inputs"}, {"createrawtransaction", 1, "outputs"}, {"createrawtransaction", 2, "locktime"},
    {"signrawtransaction", 1, "prevtxs"}, {"signrawtransaction", 2, "privkeys"}, {"sendrawtransaction", 1, "allowhighfees"},
    {"fundrawtransaction", 1, "options"}, {"gettxout", 1, "n"}, {"gettxout", 2, "include_mempool"},
    {"gettxoutproof", 0, "txids"}, {"lockunspent", 0, "unlock"}, {"lockunspent", 1, "transactions"},
    {"importprivkey", 2, "rescan"}, {"importaddress", 2, "rescan"}, {"importaddress", 3, "p2sh"},
    {"importpubkey", 2, "rescan"}, {"importmulti", 0, "requests"}, {"importmulti", 1, "options"},
    {"verifychain", 0, "checklevel"}, {"verifychain", 1, "nblocks"}, {"pruneblockchain", 0, "height"},
    {"keypoolrefill", 0, "newsize"}, {"getrawmempool", 0, "verbose"}, {"estimatefee", 0, "nblocks"},
    {"estimatepriority", 0, "nblocks"}, {"estimatesmartfee", 0, "nblocks"}, {"estimatesmartpriority", 0, "nblocks"},
    {"prioritisetransaction", 1, "priority_delta"}, {"prioritisetransaction", 2, "fee_delta"}, {"setban", 2, "bantime"},
    {"setban", 3, "absolute"}, {"setnetworkactive", 0, "state"}, {"getmempoolancestors", 1, "verbose"},
    {"getmempooldescendants", 1, "verbose"}, {"disconnectnode", 1, "nodeid"}, {"setexcessiveblock", 0, "blockSize"},
    {"echojson", 0, "arg0"}, {"echojson", 1, "arg1"}, {"echojson", 2, "arg2"}, {"echojson", 3, "arg3"},
    {"echojson", 4, "arg4"}, {"echojson", 5, "arg5"}, {"echojson", 6, "arg6"}, {"echojson", 7, "arg7"},
    {"echojson", 8, "arg8"}, {"echojson", 9, "arg9"},
};
UniValue ParseNonRFCJSONValue(const std::string& strVal) {
    UniValue jVal;
    if (!jVal.read(std::string("[") + strVal + std::string("]")) || !jVal.isArray() || jVal.size() != 1)
        throw std::runtime_error(std::string("Error parsing JSON:") + strVal);
    return jVal[0];
}
} // namespace

UniValue RPCConvertValues(const std::string& strMethod, const std::vector<std::string>& strParams) {
    UniValue params(UniValue::VARR);
    for (size_t idx = 0; idx < strParams.size(); idx++) {
        bool convert = false;
        for (const auto& c : kConvert)
            if (strMethod == c.method && (int)idx == c.idx) convert = true;
        if (!convert) params.push_back(strParams[idx]);
        else params.push_back(ParseNonRFCJSONValue(strParams[idx]));
    }
    return params;
}

UniValue RPCConvertNamedValues(const std::string& strMethod, const std::vector<std::string>& strParams) {
    UniValue params(UniValue::VOBJ);
    for (const std::string& s : strParams) {
        const size_t pos = s.find('=');
        if (pos == std::string::npos) throw std::runtime_error("No '=' in named argument '" + s + "'");
        const std::string name = s.substr(0, pos), value = s.substr(pos + 1);
        bool convert = false;
        for (const auto& c : kConvert)
            if (strMethod == c.method && name == c.name) convert = true;
        params.pushKV(name, convert ? ParseNonRFCJSONValue(value) : UniValue(value));
    }
    return params;
}

// ------------------------------------------------------------------ cookie
static const char* const COOKIEAUTH_USER = "__cookie__";
static const char* const COOKIEAUTH_FILE = ".cookie";

// -rpccookiefile: an absolute path, or one relative to the data directory (reference
// src/rpc/protocol.cpp:67 GetAuthCookieFile).
static std::string AuthCookieFile(const std::string& datadir) {
    const std::string f = gArgs.GetArg("-rpccookiefile", COOKIEAUTH_FILE);
    return !f.empty() && f[0] == '/' ? f : datadir + "/" + f;
}

bool GenerateAuthCookie(const std::string& datadir, std::string* cookie_out) {
    unsigned char rand_pwd[32];
    GetRandBytes(rand_pwd, 32);
    const std::string cookie = std::string(COOKIEAUTH_USER) + ":" + HexStr(rand_pwd, rand_pwd + 32);
    std::ofstream file(AuthCookieFile(datadir).c_str(), std::ios::out | std::ios::trunc);
    if (!file.is_open()) return false;
    file << cookie;
    file.close();
    if (cookie_out) *cookie_out = cookie;
    return true;
}
bool GetAuthCookie(const std::string& datadir, std::string* cookie_out) {
    std::ifstream file(AuthCookieFile(datadir).c_str());
    if (!file.is_open()) return false;
    std::string cookie;
    std::getline(file, cookie);
    if (cookie_out) *cookie_out = cookie;
    return true;
}
void DeleteAuthCookie(const std::string& datadir) { RemoveFile(AuthCookieFile(datadir)); }

} // namespace bcp
