// Python bindings: embedded node (chainstate + mempool + RPC dispatch) for tests and
// tools. The same CRPCTable serves the HTTP JSON-RPC server of bcpd.
#include "node/node.h"
#include "python/bind.h"
#include "rpc/server.h"
#include "util/util.h"

namespace bcp {
namespace py {

static std::unique_ptr<NodeContext> g_pynode;

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
    // Lock-order detector probe (reference DEBUG_LOCKORDER): a->b then b->a in one thread.
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
