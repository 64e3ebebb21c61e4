// RPC console command lines: nested calls, result queries and history filtering.
//
// Parity: reference src/qt/rpcconsole.cpp RPCParseCommandLine / RPCExecuteCommandLine
// (:120-400, history filter list :67) and its test src/qt/test/rpcnestedtests.cpp. The
// reference walks the line with a character state machine inside the Qt console; here a
// recursive-descent parser serves the browser GUI console (RPC `execconsole`) and tests.
//
// Syntax: `method arg arg ...` or `method(arg, arg ...)`. Arguments are separated by
// whitespace or one comma; an argument may itself be a call, `getblock(getbestblockhash())`.
// `[key]` after a call selects an object member or array element of its result. Quoting:
// '...' is literal, "..." allows \" and \\ escapes, a backslash outside quotes escapes any
// character.
#pragma once

#include "util/univalue.h"

#include <functional>
#include <string>
#include <vector>

namespace bcp {

using ConsoleExecutor = std::function<UniValue(const std::string& method, const std::vector<std::string>& args)>;

// Parses (and, when `exec` is set, executes) one console line. `result` receives the final
// result (a string result raw, anything else as indented JSON). `filtered`, when given,
// receives the line with the arguments of sensitive commands (importprivkey,
// walletpassphrase, ...) replaced by "(…)", for the console history. Throws
// std::runtime_error("Invalid Syntax" / "Invalid result query") on malformed lines; RPC
// errors from `exec` propagate unchanged.
void RPCParseCommandLine(std::string& result, const std::string& line, const ConsoleExecutor* exec,
                         std::string* filtered = nullptr);

// The executor over tableRPC: string arguments converted per method (RPCConvertValues).
UniValue ConsoleExecuteRPC(const std::string& method, const std::vector<std::string>& args);

// True for commands whose arguments never reach the console history.
bool IsSensitiveConsoleCommand(const std::string& method);

} // namespace bcp
