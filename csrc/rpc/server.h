// JSON-RPC dispatch table and helpers.
// Parity: reference src/rpc/server.{h,cpp} (CRPCTable, CRPCCommand {category, name,
// actor, okSafeMode, argNames}, named-argument transformation, help, stop, uptime
// warmup state), src/rpc/protocol.{h,cpp} (RPC error codes, JSONRPCRequest/Reply
// objects, cookie auth file ".cookie"), src/rpc/client.cpp vRPCConvertParams (CLI
// string->JSON conversion table).
#pragma once
#include "primitives/amount.h"
#include "primitives/uint256.h"
#include "util/univalue.h"

#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace bcp {

enum RPCErrorCode {
    RPC_INVALID_REQUEST = -32600,
    RPC_METHOD_NOT_FOUND = -32601,
    RPC_INVALID_PARAMS = -32602,
    RPC_INTERNAL_ERROR = -32603,
    RPC_PARSE_ERROR = -32700,
    RPC_MISC_ERROR = -1,
    RPC_FORBIDDEN_BY_SAFE_MODE = -2,
    RPC_TYPE_ERROR = -3,
    RPC_INVALID_ADDRESS_OR_KEY = -5,
    RPC_OUT_OF_MEMORY = -7,
    RPC_INVALID_PARAMETER = -8,
    RPC_DATABASE_ERROR = -20,
    RPC_DESERIALIZATION_ERROR = -22,
    RPC_VERIFY_ERROR = -25,
    RPC_VERIFY_REJECTED = -26,
    RPC_VERIFY_ALREADY_IN_CHAIN = -27,
    RPC_IN_WARMUP = -28,
    RPC_TRANSACTION_ERROR = RPC_VERIFY_ERROR,
    RPC_TRANSACTION_REJECTED = RPC_VERIFY_REJECTED,
    RPC_TRANSACTION_ALREADY_IN_CHAIN = RPC_VERIFY_ALREADY_IN_CHAIN,
    RPC_CLIENT_NOT_CONNECTED = -9,
    RPC_CLIENT_IN_INITIAL_DOWNLOAD = -10,
    RPC_CLIENT_NODE_ALREADY_ADDED = -23,
    RPC_CLIENT_NODE_NOT_ADDED = -24,
    RPC_CLIENT_NODE_NOT_CONNECTED = -29,
    RPC_CLIENT_INVALID_IP_OR_SUBNET = -30,
    RPC_CLIENT_P2P_DISABLED = -31,
    RPC_WALLET_ERROR = -4,
    RPC_WALLET_INSUFFICIENT_FUNDS = -6,
    RPC_WALLET_INVALID_ACCOUNT_NAME = -11,
    RPC_WALLET_KEYPOOL_RAN_OUT = -12,
    RPC_WALLET_UNLOCK_NEEDED = -13,
    RPC_WALLET_PASSPHRASE_INCORRECT = -14,
    RPC_WALLET_WRONG_ENC_STATE = -15,
    RPC_WALLET_ENCRYPTION_FAILED = -16,
    RPC_WALLET_ALREADY_UNLOCKED = -17,
};

// Thrown by handlers; carries the JSON error object {code, message}.
struct JSONRPCException {
    UniValue obj;
};
UniValue JSONRPCError(int code, const std::string& message);
[[noreturn]] void ThrowRPC(int code, const std::string& message);

struct JSONRPCRequest {
    UniValue id;
    std::string strMethod;
    UniValue params;
    bool fHelp = false;
    std::string URI;
    std::string authUser;
    void parse(const UniValue& valRequest);
};

typedef std::function<UniValue(const JSONRPCRequest&)> rpcfn_type;

struct CRPCCommand {
    std::string category;
    std::string name;
    rpcfn_type actor;
    bool okSafeMode;
    std::vector<std::string> argNames;
    std::string help; // usage line + description
};

class CRPCTable {
public:
    bool appendCommand(const std::string& name, const CRPCCommand& cmd);
    const CRPCCommand* operator[](const std::string& name) const;
    UniValue execute(const JSONRPCRequest& request) const;
    std::string help(const std::string& name) const;
    std::vector<std::string> listCommands() const;

private:
    std::map<std::string, CRPCCommand> mapCommands;
};
extern CRPCTable tableRPC;

// Executes a single request object or a batch array; returns the JSON reply text.
std::string JSONRPCExecute(const std::string& body, const std::string& authUser, int& httpStatus);
UniValue JSONRPCReplyObj(const UniValue& result, const UniValue& error, const UniValue& id);
UniValue JSONRPCRequestObj(const std::string& method, const UniValue& params, const UniValue& id);

// Warmup / lifecycle
void SetRPCWarmupStatus(const std::string& s);
void SetRPCWarmupFinished();
bool RPCIsInWarmup(std::string* statusOut);
void SetRPCShutdownHook(std::function<void()> f);
void RequestShutdown();
bool ShutdownRequested();
int64_t GetStartupTime();

// Argument helpers
void RPCTypeCheck(const UniValue& params, const std::vector<UniValue::VType>& typesExpected, bool fAllowNull = false);
void RPCTypeCheckArgument(const UniValue& value, UniValue::VType typeExpected);
uint256 ParseHashV(const UniValue& v, const std::string& strName);
uint256 ParseHashO(const UniValue& o, const std::string& strKey);
std::vector<unsigned char> ParseHexV(const UniValue& v, const std::string& strName);
std::vector<unsigned char> ParseHexO(const UniValue& o, const std::string& strKey);
Amount AmountFromValue(const UniValue& value);
UniValue ValueFromAmount(Amount amount);
std::string HelpExampleCli(const std::string& methodname, const std::string& args);
std::string HelpExampleRpc(const std::string& methodname, const std::string& args);

// CLI parameter conversion (string argv -> JSON typed params).
UniValue RPCConvertValues(const std::string& strMethod, const std::vector<std::string>& strParams);
UniValue RPCConvertNamedValues(const std::string& strMethod, const std::vector<std::string>& strParams);

// Cookie authentication (<datadir>/.cookie, user "__cookie__").
bool GenerateAuthCookie(const std::string& datadir, std::string* cookie_out);
bool GetAuthCookie(const std::string& datadir, std::string* cookie_out);
void DeleteAuthCookie(const std::string& datadir);

// Registration of the command groups.
void RegisterBlockchainRPCCommands(CRPCTable& t);
void RegisterMiningRPCCommands(CRPCTable& t);
void RegisterRawTransactionRPCCommands(CRPCTable& t);
void RegisterMiscRPCCommands(CRPCTable& t);
void RegisterNetRPCCommands(CRPCTable& t);
void RegisterABCRPCCommands(CRPCTable& t);
void RegisterWalletRPCCommands(CRPCTable& t);
void RegisterAllRPCCommands(CRPCTable& t);

} // namespace bcp
