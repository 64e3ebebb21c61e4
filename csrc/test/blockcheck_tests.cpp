// blockcheck_tests and validation_tests: context-free block checks, and importing a block file
// whose block is far larger than a transaction.
// Parity: reference src/test/blockcheck_tests.cpp (blockfail: no coinbase, coinbase script
// length, the block size limit reached exactly and exceeded by one transaction) and
// src/test/validation_tests.cpp (validation_load_external_block_file: a 10 x MAX_TX_SIZE block
// of empty transactions in a magic + size framed file imports without throwing).
#include "test/unittest.h"

#include "consensus/params.h"
#include "node/validation.h"
#include "util/util.h"

#include <cstdio>
#include <random>

using namespace bcp;

namespace {

uint256 RandHash(std::mt19937_64& rng) {
    uint256 h;
    for (int w = 0; w < 4; w++) {
        const uint64_t x = rng();
        memcpy(h.begin() + 8 * w, &x, 8);
    }
    return h;
}

// CheckBlock without PoW or merkle checks; the reject reason, or "" when it passes
std::string Check(Chainstate& cs, const CBlock& block) {
    block.fChecked = false;
    CValidationState state;
    const bool ok = cs.CheckBlock(block, state, false, false);
    if (ok != state.IsValid()) return "state mismatch";
    if (ok) return "";
    if (state.GetRejectCode() != REJECT_INVALID) return "bad reject code";
    return state.GetRejectReason();
}

} // namespace

TEST_CASE(blockcheck_tests, blockfail) {
    test::TestingSetup setup("regtest");
    Chainstate& cs = *setup.node->chainstate;
    std::mt19937_64 rng(1);
    CBlock block;
    CHECK_EQ(Check(cs, block), std::string("bad-cb-missing"));

    // coinbase only
    CMutableTransaction tx;
    tx.vin.resize(1);
    tx.vin[0].scriptSig.resize(10);
    tx.vout.resize(1);
    tx.vout[0].nValue = 42;
    const CTransaction coinbase(tx);
    block.vtx.push_back(MakeTransactionRef(tx));
    CHECK_EQ(Check(cs, block), std::string());

    // no coinbase: the first transaction spends something
    tx.vin[0].prevout = COutPoint(RandHash(rng), 0);
    block.vtx[0] = MakeTransactionRef(tx);
    CHECK_EQ(Check(cs, block), std::string("bad-cb-missing"));

    // coinbase script too short
    tx = CMutableTransaction(coinbase);
    tx.vin[0].scriptSig.resize(0);
    block.vtx[0] = MakeTransactionRef(tx);
    CHECK_EQ(Check(cs, block), std::string("bad-cb-length"));

    // fill up to the size limit exactly with distinct non-coinbase transactions: accepted; one
    // more: bad-blk-length
    tx = CMutableTransaction(coinbase);
    block.vtx[0] = MakeTransactionRef(tx);
    tx.vin[0].prevout = COutPoint(RandHash(rng), 0);
    const size_t txSize = GetSerializeSize(CTransaction(tx), PROTOCOL_VERSION);
    const uint64_t maxSize = cs.MaxBlockSize();
    const size_t maxTxCount = (size_t)((maxSize - 1) / txSize) - 1;
    for (size_t i = 1; i < maxTxCount; i++) {
        tx.vin[0].prevout.hash = RandHash(rng);
        block.vtx.push_back(MakeTransactionRef(tx));
    }
    CHECK_EQ(Check(cs, block), std::string());
    tx.vin[0].prevout.hash = RandHash(rng);
    block.vtx.push_back(MakeTransactionRef(tx));
    CHECK_EQ(Check(cs, block), std::string("bad-blk-length"));
}

TEST_CASE(validation_tests, load_external_block_file) {
    test::TestingSetup setup("regtest");
    Chainstate& cs = *setup.node->chainstate;
    // magic, size, then a block of empty transactions well past 2 x MAX_TX_SIZE
    const CTransaction empty;
    const size_t emptySize = GetSerializeSize(empty, PROTOCOL_VERSION);
    const size_t numTx = (size_t)(10 * MAX_TX_SIZE) / emptySize;
    CBlock block;
    for (size_t i = 0; i < numTx; i++) block.vtx.push_back(MakeTransactionRef(empty));
    const uint32_t size = (uint32_t)GetSerializeSize(block, PROTOCOL_VERSION);
    CHECK(size > 2 * MAX_TX_SIZE);
    FILE* f = tmpfile();
    REQUIRE(f != nullptr);
    fwrite(cs.Params().DiskMagic(), 1, 4, f);
    fwrite(&size, 1, 4, f);
    DataStream s(SER_DISK, PROTOCOL_VERSION);
    s << block;
    fwrite(s.data(), 1, s.size(), f);
    fseek(f, 0, SEEK_SET);
    bool threw = false;
    try {
        cs.LoadExternalBlockFile(f); // the block is invalid (no coinbase): nothing loads, nothing throws
    } catch (...) {
        threw = true;
    }
    fclose(f);
    CHECK(!threw);
    CHECK_EQ(cs.HeightNow(), 0);
}
