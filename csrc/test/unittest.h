// Minimal native unit-test harness (bin/test_bcp).
// Parity: reference src/test/ (Boost.Test suites run by test_bitcoin, fixtures in
// src/test/test_bitcoin.h:20-63: BasicTestingSetup selects chain params, TestingSetup adds an
// in-memory chainstate + mempool, TestChain100Setup mines 100 blocks to a known key).
// Suites here exercise the C++ internals directly; tests/test_unit_native.py runs every suite
// under pytest.
#pragma once
#include "consensus/params.h"
#include "keys/key.h"
#include "node/node.h"
#include "primitives/block.h"
#include "primitives/transaction.h"

#include <functional>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace bcp {
namespace test {

struct Case {
    std::string suite, name;
    std::function<void()> fn;
};
std::vector<Case>& Registry();
struct Registrar {
    Registrar(const char* suite, const char* name, std::function<void()> fn) {
        Registry().push_back({suite, name, std::move(fn)});
    }
};

struct Failure : std::runtime_error {
    using std::runtime_error::runtime_error;
};
// Non-fatal check: records a failure (the case keeps running).
void RecordFailure(const std::string& what, const char* file, int line);
[[noreturn]] void FatalFailure(const std::string& what, const char* file, int line);
// True once the running case has recorded a failure.
bool HasFailures();

template <typename A, typename B> std::string Describe(const A& a, const B& b) {
    std::ostringstream os;
    os << " [" << a << " != " << b << "]";
    return os.str();
}

// ---- fixtures
// Chain params selected for the case's lifetime (reference BasicTestingSetup).
struct BasicTestingSetup {
    explicit BasicTestingSetup(const std::string& chain = "main");
    ~BasicTestingSetup();
};
// In-memory regtest (or other chain) node: chainstate at genesis + mempool (TestingSetup).
struct TestingSetup : BasicTestingSetup {
    explicit TestingSetup(const std::string& chain = "regtest");
    ~TestingSetup();
    std::unique_ptr<NodeContext> node;
    std::string datadir;
};
// TestingSetup + 100 pre-fork blocks whose coinbases pay coinbaseKey (TestChain100Setup).
struct TestChain100Setup : TestingSetup {
    TestChain100Setup();
    // Mine a block with `txns` on the tip, coinbase paying `scriptPubKey`; returns it (connected).
    CBlock CreateAndProcessBlock(const std::vector<CMutableTransaction>& txns, const CScript& scriptPubKey);
    CKey coinbaseKey;
    std::vector<CTransaction> coinbaseTxns;
};

} // namespace test
} // namespace bcp

#define BCP_TEST_CAT2(a, b) a##b
#define BCP_TEST_CAT(a, b) BCP_TEST_CAT2(a, b)
#define TEST_CASE(suite, name)                                                                          \
    static void suite##__##name();                                                                    \
    static ::bcp::test::Registrar BCP_TEST_CAT(reg_##suite##__##name, __LINE__)(#suite, #name, suite##__##name); \
    static void suite##__##name()

#define CHECK(cond)                                                                                     \
    do {                                                                                                \
        if (!(cond)) ::bcp::test::RecordFailure("CHECK(" #cond ")", __FILE__, __LINE__);                 \
    } while (0)
#define CHECK_EQ(a, b)                                                                                  \
    do {                                                                                                \
        /* copies: a reference could dangle (e.g. std::max over temporaries) */                         \
        const auto _va = (a);                                                                           \
        const auto _vb = (b);                                                                           \
        if (!(_va == _vb))                                                                              \
            ::bcp::test::RecordFailure("CHECK_EQ(" #a ", " #b ")" + ::bcp::test::Describe(_va, _vb), __FILE__, \
                                       __LINE__);                                                       \
    } while (0)
#define REQUIRE(cond)                                                                                   \
    do {                                                                                                \
        if (!(cond)) ::bcp::test::FatalFailure("REQUIRE(" #cond ")", __FILE__, __LINE__);               \
    } while (0)
#define CHECK_THROWS(expr)                                                                              \
    do {                                                                                                \
        bool _threw = false;                                                                            \
        try {                                                                                           \
            (void)(expr);                                                                               \
        } catch (...) {                                                                                 \
            _threw = true;                                                                              \
        }                                                                                               \
        if (!_threw) ::bcp::test::RecordFailure("CHECK_THROWS(" #expr ")", __FILE__, __LINE__);         \
    } while (0)
