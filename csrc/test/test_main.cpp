// bin/test_bcp: runs the native unit suites (csrc/test/*_tests.cpp).
//   test_bcp --list            suites and cases
//   test_bcp [--suite=NAME]    run all cases (of one suite); exit status 1 on any failure
#include "test/unittest.h"

#include "consensus/params.h"
#include "consensus/pow.h"
#include "node/miner.h"
#include "node/validation.h"
#include "script/interpreter.h"
#include "util/util.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <unistd.h>

namespace bcp {
namespace test {

std::vector<Case>& Registry() {
    static std::vector<Case> r;
    return r;
}

static thread_local int g_failures = 0;
static thread_local const Case* g_current = nullptr;

void RecordFailure(const std::string& what, const char* file, int line) {
    ++g_failures;
    std::fprintf(stderr, "  FAIL %s.%s: %s (%s:%d)\n", g_current ? g_current->suite.c_str() : "?",
                 g_current ? g_current->name.c_str() : "?", what.c_str(), file, line);
}
bool HasFailures() { return g_failures != 0; }
void FatalFailure(const std::string& what, const char* file, int line) {
    RecordFailure(what, file, line);
    throw Failure(what);
}

BasicTestingSetup::BasicTestingSetup(const std::string& chain) { SelectParams(chain); }
BasicTestingSetup::~BasicTestingSetup() {}

static std::string MakeTempDir() {
    char tmpl[] = "/tmp/test_bcp_XXXXXX";
    const char* d = mkdtemp(tmpl);
    if (!d) throw std::runtime_error("mkdtemp failed");
    return d;
}

TestingSetup::TestingSetup(const std::string& chain) : BasicTestingSetup(chain) {
    datadir = MakeTempDir();
    std::string err;
    node = CreateNode(chain, datadir, /*memoryOnly=*/true, /*useGpu=*/false, err);
    if (!node) throw std::runtime_error("TestingSetup: " + err);
    SetNode(node.get());
}
TestingSetup::~TestingSetup() {
    if (node) ShutdownNode(*node);
    node.reset();
    std::string cmd = "rm -rf '" + datadir + "'";
    if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "warning: could not remove %s\n", datadir.c_str());
}

TestChain100Setup::TestChain100Setup() : TestingSetup("regtest") {
    // deterministic key (reference test_bitcoin.cpp:108 uses a fresh random key)
    std::vector<unsigned char> sec(32, 0);
    sec[31] = 0x77;
    coinbaseKey.Set(sec.begin(), sec.end(), true);
    CScript spk = CScript() << coinbaseKey.GetPubKey().Raw() << OP_CHECKSIG;
    for (int i = 0; i < COINBASE_MATURITY; i++) {
        CBlock b = CreateAndProcessBlock({}, spk);
        coinbaseTxns.push_back(*b.vtx[0]);
    }
}

CBlock TestChain100Setup::CreateAndProcessBlock(const std::vector<CMutableTransaction>& txns,
                                                const CScript& scriptPubKey) {
    Chainstate& cs = *node->chainstate;
    BlockAssembler asm_(cs, node->mempool.get());
    std::unique_ptr<CBlockTemplate> tmpl = asm_.CreateNewBlock(scriptPubKey);
    CBlock& block = tmpl->block;
    // replace the mempool selection with exactly `txns`
    block.vtx.resize(1);
    for (const CMutableTransaction& tx : txns) block.vtx.push_back(MakeTransactionRef(tx));
    unsigned extraNonce = 0;
    IncrementExtraNonce(&block, cs.Tip(), extraNonce, cs.MaxBlockSize());
    uint64_t tries = 1u << 30;
    if (!SolveBlock(block, cs.Params(), tries, false)) throw std::runtime_error("CreateAndProcessBlock: no PoW");
    auto shared = std::make_shared<const CBlock>(block);
    bool fNew = false;
    CValidationState state;
    if (!cs.ProcessNewBlock(shared, true, &fNew, &state) || cs.Tip()->GetBlockHash() != block.GetHash())
        throw std::runtime_error("CreateAndProcessBlock: block not connected: " + state.GetRejectReason());
    return block;
}

} // namespace test
} // namespace bcp

int main(int argc, char** argv) {
    using namespace bcp::test;
    std::string only;
    bool list = false;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--list")) list = true;
        else if (!std::strncmp(argv[i], "--suite=", 8)) only = argv[i] + 8;
        else {
            std::fprintf(stderr, "usage: %s [--list] [--suite=NAME]\n", argv[0]);
            return 2;
        }
    }
    if (list) {
        std::map<std::string, int> n;
        for (const Case& c : Registry()) n[c.suite]++;
        for (const auto& kv : n) std::printf("%s %d\n", kv.first.c_str(), kv.second);
        return 0;
    }
    int ran = 0, failed = 0;
    for (const Case& c : Registry()) {
        if (!only.empty() && c.suite != only) continue;
        g_current = &c;
        g_failures = 0;
        try {
            c.fn();
        } catch (const Failure&) {
        } catch (const std::exception& e) {
            RecordFailure(std::string("uncaught exception: ") + e.what(), __FILE__, __LINE__);
        }
        ran++;
        if (g_failures) failed++;
        std::printf("%s %s.%s\n", g_failures ? "FAIL" : "ok  ", c.suite.c_str(), c.name.c_str());
        std::fflush(stdout);
    }
    std::printf("%d cases, %d failed\n", ran, failed);
    return ran == 0 ? 2 : (failed ? 1 : 0);
}
