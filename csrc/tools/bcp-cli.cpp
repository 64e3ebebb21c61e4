// bcp-cli: command-line JSON-RPC client (reference src/bitcoin-cli.cpp: -rpcconnect,
// -rpcport, -rpcuser/-rpcpassword or cookie auth, -rpcwait, -named, -stdin,
// -rpcclienttimeout; result printing: strings raw, other JSON pretty; error -> exit code
// abs(code)).
#include "consensus/params.h"
#include "rpc/httpserver.h"
#include "rpc/server.h"
#include "util/univalue.h"
#include "util/util.h"

#include <cstdio>
#include <iostream>

using namespace bcp;

static const char* const kHelp =
    "Usage:\n"
    "  bcp-cli [options] <command> [params]      Send command to bcpd\n"
    "  bcp-cli [options] -named <command> [name=value] ...\n"
    "  bcp-cli [options] help                    List commands\n\n"
    "Options:\n"
    "  -conf=<file>          Specify configuration file (default: bitcoincashplus.conf)\n"
    "  -datadir=<dir>        Specify data directory\n"
    "  -testnet / -regtest   Chain selection\n"
    "  -named                Pass named instead of positional arguments\n"
    "  -rpcconnect=<ip>      Send commands to node running on <ip> (default: 127.0.0.1)\n"
    "  -rpcport=<port>       Connect to JSON-RPC on <port>\n"
    "  -rpcwait              Wait for RPC server to start\n"
    "  -rpcuser=<user>       Username for JSON-RPC connections\n"
    "  -rpcpassword=<pw>     Password for JSON-RPC connections\n"
    "  -rpcclienttimeout=<n> Timeout in seconds during HTTP requests, or 0 for no timeout (default: 900)\n"
    "  -stdin                Read extra arguments from standard input, one per line\n"
    "  -rpcwallet=<name>     Send RPC for non-default wallet on RPC server\n";

int main(int argc, char* argv[]) {
    // split options (leading -x) from the command and its params
    int first = 1;
    while (first < argc && argv[first][0] == '-' && !(argv[first][1] >= '0' && argv[first][1] <= '9')) first++;
    gArgs.ParseParameters(first, argv);
    if (argc < 2 || gArgs.IsArgSet("-?") || gArgs.IsArgSet("-h") || gArgs.IsArgSet("-help")) {
        printf("%s", kHelp);
        return argc < 2 ? 1 : 0;
    }
    if (gArgs.IsArgSet("-version")) {
        printf("%s RPC client version %s\n", CLIENT_NAME, FormatFullVersion().c_str());
        return 0;
    }
    const std::string datadirBase = gArgs.GetArg("-datadir", GetDefaultDataDir());
    SetDataDir(datadirBase);
    gArgs.ReadConfigFile(datadirBase + "/" + gArgs.GetArg("-conf", "bitcoincashplus.conf"));
    std::string chain;
    try {
        chain = gArgs.GetChainName();
    } catch (const std::exception& e) {
        fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    SelectParams(chain);
    if (gArgs.GetBoolArg("-rpcssl", false)) { // reference src/bitcoin-cli.cpp:143
        fprintf(stderr, "Error: SSL mode for RPC (-rpcssl) is no longer supported.\n");
        return 1;
    }

    std::vector<std::string> args(argv + first, argv + argc);
    if (gArgs.GetBoolArg("-stdin", false)) {
        std::string line;
        while (std::getline(std::cin, line)) args.push_back(line);
    }
    if (args.empty()) {
        fprintf(stderr, "error: too few parameters (need at least command)\n");
        return 1;
    }
    const std::string method = args[0];
    args.erase(args.begin());

    UniValue params;
    try {
        params = gArgs.GetBoolArg("-named", false) ? RPCConvertNamedValues(method, args) : RPCConvertValues(method, args);
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }

    std::string auth;
    if (gArgs.GetArg("-rpcpassword", "").empty()) {
        if (!GetAuthCookie(GetDataDir(true), &auth)) {
            fprintf(stderr, "error: Could not locate RPC credentials. No authentication cookie could be found, and "
                            "RPC password is not set.\n");
            return 1;
        }
    } else {
        auth = gArgs.GetArg("-rpcuser", "") + ":" + gArgs.GetArg("-rpcpassword", "");
    }
    const std::string host = gArgs.GetArg("-rpcconnect", "127.0.0.1");
    const int port = (int)gArgs.GetArg("-rpcport", (int64_t)Params().GetRPCPort());
    std::string path = "/";
    if (gArgs.IsArgSet("-rpcwallet")) path = "/wallet/" + gArgs.GetArg("-rpcwallet", "");
    const std::string body = JSONRPCRequestObj(method, params, UniValue(1)).write() + "\n";
    const int timeout = (int)gArgs.GetArg("-rpcclienttimeout", (int64_t)900);
    const bool wait = gArgs.GetBoolArg("-rpcwait", false);

    for (;;) {
        int status = 0;
        std::string response;
        if (!HTTPPost(host, port, path, auth, body, status, response, timeout)) {
            if (wait) {
                MilliSleep(1000);
                continue;
            }
            fprintf(stderr, "error: couldn't connect to server: unknown (code -1)\n"
                            "(make sure server is running and you are connecting to the correct RPC port)\n");
            return 1;
        }
        if (status == 401) {
            fprintf(stderr, "error: incorrect rpcuser or rpcpassword (authorization failed)\n");
            return 1;
        }
        UniValue reply;
        if (!reply.read(response) || !reply.isObject()) {
            if (status >= 400) {
                fprintf(stderr, "error: server returned HTTP error %d\n", status);
                return 1;
            }
            fprintf(stderr, "error: couldn't parse reply from server\n");
            return 1;
        }
        const UniValue& error = find_value(reply, "error");
        const UniValue& result = find_value(reply, "result");
        if (!error.isNull()) {
            const int code = find_value(error, "code").isNum() ? find_value(error, "code").get_int() : -1;
            if (wait && code == RPC_IN_WARMUP) {
                MilliSleep(1000);
                continue;
            }
            const UniValue& msg = find_value(error, "message");
            fprintf(stderr, "error code: %d\nerror message:\n%s\n", code, msg.isStr() ? msg.get_str().c_str() : error.write().c_str());
            return code < 0 ? -code : (code ? code : 1);
        }
        if (result.isNull()) return 0;
        if (result.isStr())
            printf("%s\n", result.get_str().c_str());
        else
            printf("%s\n", result.write(2).c_str());
        return 0;
    }
}
