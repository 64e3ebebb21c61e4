// Python bindings: embedded node (chainstate + mempool + RPC dispatch) for tests and
// tools. The same CRPCTable serves the HTTP JSON-RPC server of bcpd.
#include "node/node.h"
#include "node/ui_interface.h"
#include "python/bind.h"
#include "rpc/console.h"
#include "rpc/server.h"
#include "util/checkqueue.h"
#include "util/cuckoocache.h"
#include "util/indirectmap.h"
#include "util/limitedmap.h"
#include "util/memusage.h"
#include "util/util.h"

#include <sys/resource.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <thread>
#include <map>

namespace bcp {
namespace py {

static std::unique_ptr<NodeContext> g_pynode;

// UI signal observer for tests: counts emissions per signal and remembers the last
// values (connected on ui_track_start, removed on ui_track_stop).
struct UITracker {
    std::mutex m;
    std::map<std::string, int> counts;
    std::vector<std::string> initMessages;
    int lastTipHeight = -1, lastHeaderHeight = -1, lastConnections = -1, lastProgress = -1;
    std::vector<std::pair<std::function<void()>, int>> conns;
    void bump(const char* name) {
        std::lock_guard<std::mutex> l(m);
        counts[name]++;
    }
};
static UITracker g_ui;

// Deterministic key stream for the cache simulations (splitmix64).
struct SimRng {
    uint64_t x;
    uint64_t next() {
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    uint256 key() {
        uint256 k;
        for (int i = 0; i < 4; ++i) {
            const uint64_t v = next();
            memcpy(k.begin() + 8 * i, &v, 8);
        }
        return k;
    }
};

// Cache behaviour simulations mirroring reference src/test/cuckoocache_tests.cpp.
static double CuckooHitRate(size_t megabytes, double load) {
    CuckooHashSet set;
    const size_t cap = set.setup_bytes(megabytes << 20);
    const size_t n = (size_t)(load * cap);
    SimRng r{1};
    std::vector<uint256> keys(n);
    for (auto& k : keys) k = r.key();
    for (auto& k : keys) set.insert(k);
    size_t hits = 0;
    for (auto& k : keys) hits += set.contains(k, false);
    return (double)hits / (double)n;
}

// Insert 1x capacity; erase the first quarter; insert half a capacity more. Returns
// (hit rate of erased quarter, of the un-erased second quarter, of the fresh half).
static std::vector<double> CuckooErase(size_t megabytes) {
    CuckooHashSet set;
    const size_t cap = set.setup_bytes(megabytes << 20);
    SimRng r{2};
    std::vector<uint256> keys(cap + cap / 2);
    for (auto& k : keys) k = r.key();
    for (size_t i = 0; i < cap; ++i) set.insert(keys[i]);
    for (size_t i = 0; i < cap / 2; ++i) set.contains(keys[i], true);
    for (size_t i = cap; i < keys.size(); ++i) set.insert(keys[i]);
    size_t erased = 0, stale = 0, fresh = 0;
    for (size_t i = 0; i < cap / 2; ++i) erased += set.contains(keys[i], false);
    for (size_t i = cap / 2; i < cap; ++i) stale += set.contains(keys[i], false);
    for (size_t i = cap; i < keys.size(); ++i) fresh += set.contains(keys[i], false);
    return {erased / double(cap / 2), stale / double(cap / 2), fresh / double(keys.size() - cap)};
}

// Sliding window of "blocks": each inserts block_size keys and later consumes the
// first and last quarter of them. Returns (min window hit rate, fraction of windows
// under 99.9%).
static std::vector<double> CuckooGenerations(size_t megabytes, double load) {
    CuckooHashSet set;
    const size_t cap = set.setup_bytes(megabytes << 20);
    const uint32_t BLOCK = 10000, WINDOW = 60, POP = (BLOCK / WINDOW) / 2;
    const size_t total = (size_t)(load * cap) / BLOCK;
    SimRng r{3};
    std::deque<std::vector<uint256>> window;
    double minHit = 1.0;
    size_t loose = 0;
    for (size_t b = 0; b < total; ++b) {
        if (window.size() == WINDOW) window.pop_front();
        std::vector<uint256> ins(BLOCK), reads;
        for (auto& k : ins) k = r.key();
        reads.insert(reads.end(), ins.begin(), ins.begin() + BLOCK / 4);
        reads.insert(reads.end(), ins.end() - BLOCK / 4, ins.end());
        for (auto& k : ins) set.insert(k);
        window.push_back(std::move(reads));
        size_t count = 0;
        for (auto& w : window)
            for (uint32_t j = 0; j < POP; ++j) {
                count += set.contains(w.back(), true);
                w.pop_back();
            }
        const double hit = (double)count / double(window.size() * POP);
        minHit = std::min(minHit, hit);
        loose += hit < 0.999;
    }
    return {minHit, (double)loose / (double)total};
}

void bind_node(pyb::module_& m) {
    m.def(
        "node_start",
        [](const std::string& chain, const std::string& datadir, bool memory, bool gpu,
           const std::vector<std::string>& args) {
            if (g_pynode) throw std::runtime_error("node already running");
            std::vector<const char*> argv{"bcp"};
            for (const auto& a : args) argv.push_back(a.c_str());
            gArgs.ParseParameters((int)argv.size(), argv.data());
            if (gArgs.GetBoolArg("-printtoconsole", false)) LogInit("", true);
            for (const auto& c : gArgs.GetArgs("-debug")) LogEnableCategory(c);
            RegisterAllRPCCommands(tableRPC);
            std::string err;
            {
                pyb::gil_scoped_release nogil;
                g_pynode = CreateNode(chain, datadir, memory, gpu, err);
            }
            if (!g_pynode) throw std::runtime_error("node init failed: " + err);
            SetNode(g_pynode.get());
            SetRPCWarmupFinished();
        },
        pyb::arg("chain") = "regtest", pyb::arg("datadir"), pyb::arg("memory") = false, pyb::arg("gpu") = false,
        pyb::arg("args") = std::vector<std::string>());
    m.def("node_stop", []() {
        if (!g_pynode) return;
        pyb::gil_scoped_release nogil;
        ShutdownNode(*g_pynode);
        g_pynode.reset();
    });
    m.def("node_running", []() { return (bool)g_pynode; });
    // CheckQueue exercise (reference src/test/checkqueue_tests.cpp): publishes `total` jobs in
    // steps of `step` with `idle_ms` pauses in between; returns (sum of run indices, jobs run,
    // jobs run by workers, process CPU seconds spent while the session sat idle).
    m.def(
        "checkqueue_run",
        [](int workers, size_t total, size_t step, int idle_ms) {
            pyb::gil_scoped_release rel;
            auto res = std::make_tuple((uint64_t)0, (uint64_t)0, (size_t)0, 0.0);
            CheckQueue q(workers);
            std::atomic<uint64_t> sum{0}, cnt{0};
            auto cpu = []() {
                struct rusage ru;
                getrusage(RUSAGE_SELF, &ru);
                return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
            };
            double idleCpu = 0;
            for (int rep = 0; rep < 2; rep++) { // two sessions on the same queue
                q.Begin([&](size_t k) {
                    sum += k;
                    cnt++;
                });
                for (size_t p = 0; p < total;) {
                    p = std::min(total, p + step);
                    q.Publish(p);
                    if (idle_ms > 0) {
                        const double c0 = cpu();
                        std::this_thread::sleep_for(std::chrono::milliseconds(idle_ms));
                        idleCpu += cpu() - c0;
                    }
                }
                q.Complete();
            }
            res = std::make_tuple((uint64_t)sum, (uint64_t)cnt, q.WorkerJobs(), idleCpu);
            return res; // converted to a Python tuple after the GIL is re-acquired
        },
        pyb::arg("workers"), pyb::arg("total"), pyb::arg("step"), pyb::arg("idle_ms") = 0);
    // Lock-order detector probe (reference DEBUG_LOCKORDER): a->b then b->a in one thread.
    m.def("ui_track_start", []() {
        {
            std::lock_guard<std::mutex> l(g_ui.m);
            g_ui.counts.clear();
            g_ui.initMessages.clear();
        }
        auto add = [](auto& sig, auto fn) {
            const int id = sig.connect(fn);
            g_ui.conns.emplace_back([&sig, id] { sig.disconnect(id); }, id);
        };
        add(uiInterface.NotifyBlockTip, [](bool, const CBlockIndex* p) {
            g_ui.bump("NotifyBlockTip");
            g_ui.lastTipHeight = p ? p->nHeight : -1;
        });
        add(uiInterface.NotifyHeaderTip, [](bool, const CBlockIndex* p) {
            g_ui.bump("NotifyHeaderTip");
            g_ui.lastHeaderHeight = p ? p->nHeight : -1;
        });
        add(uiInterface.InitMessage, [](const std::string& s) {
            g_ui.bump("InitMessage");
            std::lock_guard<std::mutex> l(g_ui.m);
            g_ui.initMessages.push_back(s);
        });
        add(uiInterface.ShowProgress, [](const std::string&, int p) {
            g_ui.bump("ShowProgress");
            g_ui.lastProgress = p;
        });
        add(uiInterface.NotifyNumConnectionsChanged, [](int n) {
            g_ui.bump("NotifyNumConnectionsChanged");
            g_ui.lastConnections = n;
        });
        add(uiInterface.NotifyNetworkActiveChanged, [](bool) { g_ui.bump("NotifyNetworkActiveChanged"); });
        add(uiInterface.BannedListChanged, []() { g_ui.bump("BannedListChanged"); });
        add(uiInterface.NotifyAlertChanged, []() { g_ui.bump("NotifyAlertChanged"); });
        add(uiInterface.LoadWallet, [](CWallet*) { g_ui.bump("LoadWallet"); });
        add(uiInterface.ThreadSafeMessageBox, [](const std::string&, const std::string&, unsigned) {
            g_ui.bump("ThreadSafeMessageBox");
            return true;
        });
    });
    m.def("ui_track_stop", []() {
        for (auto& c : g_ui.conns) c.first();
        g_ui.conns.clear();
    });
    m.def("ui_track_counts", []() {
        std::lock_guard<std::mutex> l(g_ui.m);
        pyb::dict d;
        for (auto& kv : g_ui.counts) d[pyb::str(kv.first)] = kv.second;
        d["lastTipHeight"] = g_ui.lastTipHeight;
        d["lastHeaderHeight"] = g_ui.lastHeaderHeight;
        d["lastProgress"] = g_ui.lastProgress;
        d["initMessages"] = g_ui.initMessages;
        return d;
    });
    m.def("ui_init_message", [](const std::string& s) { uiInterface.InitMessage(s); });
    m.def("ui_init_error", [](const std::string& s) { return InitError(s); });
    // container utilities (reference limitedmap.h / indirectmap.h / memusage.h), exposed for tests
    using LMap = limitedmap<int64_t, int64_t>;
    pyb::class_<LMap>(m, "LimitedMap")
        .def(pyb::init<size_t>())
        .def("insert", [](LMap& l, int64_t k, int64_t v) { l.insert({k, v}); })
        .def("erase", [](LMap& l, int64_t k) { l.erase(k); })
        .def("update", [](LMap& l, int64_t k, int64_t v) {
            auto it = l.find(k);
            if (it == l.end()) throw pyb::key_error("no such key");
            l.update(it, v);
        })
        .def("get", [](const LMap& l, int64_t k) -> pyb::object {
            auto it = l.find(k);
            return it == l.end() ? pyb::object(pyb::none()) : pyb::object(pyb::int_(it->second));
        })
        .def("set_max_size", [](LMap& l, size_t n) { return l.max_size(n); })
        .def("__len__", &LMap::size)
        .def("keys", [](const LMap& l) {
            std::vector<int64_t> k;
            for (const auto& kv : l) k.push_back(kv.first);
            return k;
        });
    m.def("indirectmap_probe", [](const std::vector<int64_t>& values) {
        // keys live in `values`; the map orders and finds them by value, not by address
        indirectmap<int64_t, size_t> im;
        for (size_t i = 0; i < values.size(); ++i) im.insert(std::make_pair(&values[i], i));
        std::vector<int64_t> order;
        for (const auto& kv : im) order.push_back(*kv.first);
        const int64_t probe = values.empty() ? 0 : values[0];
        auto it = im.find(probe);
        return pyb::make_tuple(order, it == im.end() ? -1 : (int64_t)it->second, (int64_t)im.count(probe));
    });
    m.def("malloc_usage", &memusage::MallocUsage);
    m.def("memusage_vector_u8", [](size_t cap) {
        std::vector<unsigned char> v;
        v.reserve(cap);
        return memusage::DynamicUsage(v);
    });
    m.def("cuckoo_hit_rate", &CuckooHitRate, pyb::arg("megabytes"), pyb::arg("load"));
    m.def("cuckoo_erase", &CuckooErase, pyb::arg("megabytes"));
    m.def("cuckoo_generations", &CuckooGenerations, pyb::arg("megabytes") = 32, pyb::arg("load") = 10.0);
    m.def("lockorder_probe", []() {
        const uint64_t before = LockOrderViolations();
        const bool was = LockOrderChecking();
        SetLockOrderChecking(true, false);
        CCriticalSection a("probe.a"), b("probe.b");
        {
            std::lock_guard<CCriticalSection> la(a);
            std::lock_guard<CCriticalSection> lb(b);
        }
        const uint64_t mid = LockOrderViolations();
        {
            std::lock_guard<CCriticalSection> lb(b);
            std::lock_guard<CCriticalSection> la(a);
        }
        SetLockOrderChecking(was, true);
        return pyb::make_tuple(mid - before, LockOrderViolations() - before);
    });
    // RPC console line parser with a Python executor: executor(method, [str args]) returns the
    // call's result as JSON text (None: parse and filter only). Returns (result, filtered).
    m.def(
        "console_parse",
        [](const std::string& line, pyb::object executor) {
            std::string result, filtered;
            ConsoleExecutor exec = [&](const std::string& method, const std::vector<std::string>& args) {
                const std::string js = executor(method, args).cast<std::string>();
                UniValue v;
                if (!v.read(js)) throw std::invalid_argument("executor must return JSON");
                return v;
            };
            RPCParseCommandLine(result, line, executor.is_none() ? nullptr : &exec, &filtered);
            return pyb::make_tuple(result, filtered);
        },
        pyb::arg("line"), pyb::arg("executor") = pyb::none());
    // JSON in, JSON out: {"result": ..., "error": ...}
    m.def("rpc_json", [](const std::string& method, const std::string& paramsJson) {
        std::string out;
        {
            pyb::gil_scoped_release nogil;
            UniValue params;
            if (!params.read(paramsJson)) throw std::invalid_argument("params must be JSON");
            UniValue req(UniValue::VOBJ);
            req.pushKV("method", method);
            req.pushKV("params", params);
            req.pushKV("id", 1);
            int status;
            out = JSONRPCExecute(req.write(), "python", status);
        }
        return out;
    });
    m.def("set_mock_time", &SetMockTime);
}

} // namespace py
} // namespace bcp
