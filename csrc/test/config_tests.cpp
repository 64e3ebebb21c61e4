// config_tests: the excessive block size setting refuses anything up to the legacy 1 MB limit
// and keeps its previous value, accepts 1 MB + 1 and larger, and can be lowered again; the
// node's chain parameters are the selected ones.
// Parity: reference src/test/config_tests.cpp (max_block_size, chain_params), with the
// reference's GlobalConfig replaced by the Chainstate that holds the setting here.
#include "test/unittest.h"

#include "node/validation.h"

using namespace bcp;

TEST_CASE(config_tests, max_block_size) {
    bcp::test::TestingSetup setup("regtest");
    Chainstate& cs = *setup.node->chainstate;
    CHECK(!cs.SetMaxBlockSize(0));
    CHECK(!cs.SetMaxBlockSize(12345));
    CHECK(!cs.SetMaxBlockSize(LEGACY_MAX_BLOCK_SIZE - 1));
    CHECK(!cs.SetMaxBlockSize(LEGACY_MAX_BLOCK_SIZE));
    CHECK(cs.SetMaxBlockSize(LEGACY_MAX_BLOCK_SIZE + 1));
    CHECK_EQ(cs.MaxBlockSize(), LEGACY_MAX_BLOCK_SIZE + 1);
    CHECK(cs.SetMaxBlockSize(2 * ONE_MEGABYTE));
    CHECK_EQ(cs.MaxBlockSize(), 2 * ONE_MEGABYTE);
    CHECK(cs.SetMaxBlockSize(8 * ONE_MEGABYTE));
    CHECK_EQ(cs.MaxBlockSize(), 8 * ONE_MEGABYTE);
    CHECK(!cs.SetMaxBlockSize(54321)); // refused: unchanged
    CHECK_EQ(cs.MaxBlockSize(), 8 * ONE_MEGABYTE);
    CHECK(cs.SetMaxBlockSize(7 * ONE_MEGABYTE));
    CHECK_EQ(cs.MaxBlockSize(), 7 * ONE_MEGABYTE);
    CHECK(cs.SetMaxBlockSize(ONE_MEGABYTE + 1));
    CHECK_EQ(cs.MaxBlockSize(), ONE_MEGABYTE + 1);
}

TEST_CASE(config_tests, chain_params) {
    for (const char* chain : {"main", "test", "regtest"}) {
        bcp::test::BasicTestingSetup setup(chain);
        CHECK_EQ(Params().NetworkIDString(), std::string(chain));
    }
}
