#include "util/sync.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <cstdlib>
#include <map>
#include <set>
#include <vector>

namespace bcp {
namespace detail {
std::atomic<bool> g_lockorder{false};
}

namespace {
struct Held {
    const void* cs;
    const char* name;
};
thread_local std::vector<Held> t_stack;
std::mutex g_ordersMutex;
std::map<std::pair<const void*, const void*>, std::pair<std::string, std::string>> g_orders; // (a,b) seen: a then b
std::atomic<bool> g_abort{true};
std::atomic<uint64_t> g_violations{0};
} // namespace

void SetLockOrderChecking(bool on, bool abortOnDeadlock) {
    g_abort = abortOnDeadlock;
    detail::g_lockorder = on;
}
bool LockOrderChecking() { return detail::g_lockorder.load(); }
uint64_t LockOrderViolations() { return g_violations.load(); }

void detail::EnterCritical(const void* cs, const char* name) {
    bool reentrant = false;
    for (const Held& h : t_stack)
        if (h.cs == cs) reentrant = true;
    if (!reentrant) {
        std::lock_guard<std::mutex> l(g_ordersMutex);
        for (const Held& h : t_stack) {
            const auto rev = g_orders.find({cs, h.cs});
            if (rev != g_orders.end()) {
                g_violations++;
                std::string msg = "POTENTIAL DEADLOCK DETECTED\nPrevious lock order was:\n  " + rev->second.first +
                                  " (" + strprintf("%p", rev->first.first) + ")\n  " + rev->second.second + " (" +
                                  strprintf("%p", rev->first.second) + ")\nCurrent lock order is:\n";
                for (const Held& x : t_stack) msg += "  " + std::string(x.name) + strprintf(" (%p)\n", x.cs);
                msg += "  " + std::string(name) + strprintf(" (%p)\n", cs);
                LogPrintf("%s", msg.c_str());
                fprintf(stderr, "%s", msg.c_str());
                if (g_abort) abort();
            }
            g_orders.emplace(std::make_pair(h.cs, cs), std::make_pair(std::string(h.name), std::string(name)));
        }
    }
    t_stack.push_back({cs, name});
}

void detail::LeaveCritical(const void* cs) {
    for (auto it = t_stack.rbegin(); it != t_stack.rend(); ++it)
        if (it->cs == cs) {
            t_stack.erase(std::next(it).base());
            return;
        }
}

bool detail::HoldsLock(const void* cs) {
    for (const Held& h : t_stack)
        if (h.cs == cs) return true;
    return false;
}

void AssertLockHeldImpl(const CCriticalSection& cs, const char* file, int line) {
    if (!LockOrderChecking() || detail::HoldsLock(&cs)) return;
    fprintf(stderr, "Assertion failed: lock %s not held in %s:%d\n", cs.Name(), file, line);
    abort();
}

void AssertLockNotHeldImpl(const CCriticalSection& cs, const char* file, int line) {
    if (!LockOrderChecking() || !detail::HoldsLock(&cs)) return;
    fprintf(stderr, "Assertion failed: lock %s held in %s:%d\n", cs.Name(), file, line);
    abort();
}

} // namespace bcp
