// Warning board + safe mode; see warnings.h.
#include "node/warnings.h"

#include "rpc/server.h"
#include "util/util.h"

#include <mutex>

namespace bcp {

namespace {
std::mutex g_mu;
std::string g_misc;
bool g_large_fork = false;
bool g_large_invalid = false;
} // namespace

void SetMiscWarning(const std::string& warning) {
    std::lock_guard<std::mutex> l(g_mu);
    g_misc = warning;
}
std::string GetMiscWarning() {
    std::lock_guard<std::mutex> l(g_mu);
    return g_misc;
}
void SetLargeWorkForkFound(bool on) {
    std::lock_guard<std::mutex> l(g_mu);
    g_large_fork = on;
}
bool GetLargeWorkForkFound() {
    std::lock_guard<std::mutex> l(g_mu);
    return g_large_fork;
}
void SetLargeWorkInvalidChainFound(bool on) {
    std::lock_guard<std::mutex> l(g_mu);
    g_large_invalid = on;
}
bool GetLargeWorkInvalidChainFound() {
    std::lock_guard<std::mutex> l(g_mu);
    return g_large_invalid;
}

std::string GetWarnings(const std::string& strFor) {
    std::string status, rpc;
    if (gArgs.GetBoolArg("-testsafemode", false)) status = rpc = "testsafemode enabled";
    {
        std::lock_guard<std::mutex> l(g_mu);
        // later assignments take precedence (most severe last)
        if (!g_misc.empty()) status = g_misc;
        if (g_large_fork) {
            status = rpc = "Warning: The network does not appear to fully agree! Some miners appear to be "
                           "experiencing issues.";
        } else if (g_large_invalid) {
            status = rpc = "Warning: We do not appear to fully agree with our peers! You may need to upgrade, "
                           "or other nodes may need to upgrade.";
        }
    }
    if (strFor == "rpc") return rpc;
    return status; // "statusbar" and "gui"
}

void ObserveSafeMode() {
    const std::string warning = GetWarnings("rpc");
    if (!warning.empty() && !gArgs.GetBoolArg("-disablesafemode", false))
        ThrowRPC(RPC_FORBIDDEN_BY_SAFE_MODE, "Safe mode: " + warning);
}

} // namespace bcp
