// undo_tests: a block's coin changes applied with their undo record, then reverted with
// ApplyBlockUndo: the coinbase and the spending transaction's outputs disappear, the spent
// coin comes back, and the view's best block returns to the block's parent.
// Parity: reference src/test/undo_tests.cpp (connect_utxo_extblock).
#include "test/unittest.h"

#include "node/coins.h"
#include "node/validation.h"

using namespace bcp;
using bcp::test::BasicTestingSetup;

namespace {

void UpdateUTXOSet(const CBlock& block, CCoinsViewCache& view, CBlockUndo& blockundo, int nHeight) {
    UpdateCoins(*block.vtx[0], view, nHeight);
    for (size_t i = 1; i < block.vtx.size(); i++) {
        blockundo.vtxundo.push_back(CTxUndo());
        UpdateCoins(*block.vtx[i], view, blockundo.vtxundo.back(), nHeight);
    }
    view.SetBestBlock(block.GetHash());
}

bool HasSpendableCoin(const CCoinsViewCache& view, const uint256& txid) {
    return !view.AccessCoin(COutPoint(txid, 0)).IsSpent();
}

} // namespace

TEST_CASE(undo_tests, connect_utxo_extblock) {
    BasicTestingSetup setup("main");
    CCoinsView coinsDummy;
    CCoinsViewCache view(&coinsDummy);
    CBlock block;
    block.hashPrevBlock = GetRandHash();
    view.SetBestBlock(block.hashPrevBlock);

    // a coinbase and one transaction spending an existing coin
    CMutableTransaction tx;
    tx.vin.resize(1);
    tx.vin[0].scriptSig.resize(10);
    tx.vout.resize(1);
    tx.vout[0].nValue = 42;
    const CTransaction coinbaseTx(tx);
    block.vtx.resize(2);
    block.vtx[0] = MakeTransactionRef(tx);

    tx.vout[0].scriptPubKey = CScript() << OP_TRUE;
    tx.vin[0].prevout = COutPoint(GetRandHash(), 0);
    tx.vin[0].nSequence = CTxIn::SEQUENCE_FINAL;
    tx.vin[0].scriptSig.resize(0);
    tx.nVersion = 2;
    const CTransaction prevTx0(tx);
    AddCoins(view, prevTx0, 100);

    tx.vin[0].prevout = COutPoint(prevTx0.GetHash(), 0);
    const CTransaction tx0(tx);
    block.vtx[1] = MakeTransactionRef(tx0);

    CBlockUndo blockundo;
    UpdateUTXOSet(block, view, blockundo, 123456);
    CHECK(view.GetBestBlock() == block.GetHash());
    CHECK(HasSpendableCoin(view, coinbaseTx.GetHash()));
    CHECK(HasSpendableCoin(view, tx0.GetHash()));
    CHECK(!HasSpendableCoin(view, prevTx0.GetHash()));

    CBlockIndex pindex;
    pindex.nHeight = 123456;
    CHECK_EQ((int)ApplyBlockUndo(blockundo, block, &pindex, view), (int)DISCONNECT_OK);
    CHECK(view.GetBestBlock() == block.hashPrevBlock);
    CHECK(!HasSpendableCoin(view, coinbaseTx.GetHash()));
    CHECK(!HasSpendableCoin(view, tx0.GetHash()));
    CHECK(HasSpendableCoin(view, prevTx0.GetHash()));
}

TEST_CASE(undo_tests, inconsistent_undo_fails) {
    // an undo record whose size does not match the block is refused, not applied
    BasicTestingSetup setup("main");
    CCoinsView coinsDummy;
    CCoinsViewCache view(&coinsDummy);
    CBlock block;
    CMutableTransaction cb;
    cb.vin.resize(1);
    cb.vout.resize(1);
    block.vtx.push_back(MakeTransactionRef(cb));
    CBlockUndo undo;
    undo.vtxundo.resize(1);
    CBlockIndex pindex;
    CHECK_EQ((int)ApplyBlockUndo(undo, block, &pindex, view), (int)DISCONNECT_FAILED);
}
