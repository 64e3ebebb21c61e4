// accounting_tests: order positions of wallet transactions and accounting entries across
// ReorderTransactions: records without a position (-1, from wallets that predate ordering) are
// slotted in by time and the ordered ones shift past them, for transactions and "move" entries
// added in every interleaving of the reference scenario.
// Parity: reference src/wallet/test/accounting_tests.cpp (acc_orderupgrade).
#include "test/unittest.h"

#include "wallet/wallet.h"

#include <map>

using namespace bcp;

namespace {

void GetResults(CWallet& w, std::map<int64_t, CAccountingEntry>& results) {
    results.clear();
    CHECK(w.ReorderTransactions());
    for (const CAccountingEntry& ae : w.laccentries)
        if (ae.strAccount.empty()) results[ae.nOrderPos] = ae;
}

CWalletTx* Add(CWallet& w, CWalletTx& wtx) {
    w.AddToWallet(wtx);
    return &w.mapWallet[wtx.GetHash()];
}

void Rehash(CWalletTx& wtx) { // a different lock time: a different hash
    CMutableTransaction tx(*wtx.tx);
    --tx.nLockTime;
    wtx.tx = MakeTransactionRef(std::move(tx));
}

} // namespace

TEST_CASE(accounting_tests, acc_orderupgrade) {
    CWallet w("test", "", true);
    WalletLock l(w);
    std::vector<CWalletTx*> vpwtx;
    CWalletTx wtx(&w, MakeTransactionRef(CMutableTransaction()));
    CAccountingEntry ae;
    std::map<int64_t, CAccountingEntry> results;

    ae.strAccount = "";
    ae.nCreditDebit = 1;
    ae.nTime = 1333333333;
    ae.strOtherAccount = "b";
    ae.strComment = "";
    w.AddAccountingEntry(ae);

    wtx.mapValue["comment"] = "z";
    vpwtx.push_back(Add(w, wtx));
    vpwtx[0]->nTimeReceived = 1333333335;
    vpwtx[0]->nOrderPos = -1;

    ae.nTime = 1333333336;
    ae.strOtherAccount = "c";
    w.AddAccountingEntry(ae);

    GetResults(w, results);
    CHECK_EQ(w.nOrderPosNext, (int64_t)3);
    CHECK_EQ(results.size(), (size_t)2);
    CHECK_EQ(results[0].nTime, (int64_t)1333333333);
    CHECK(results[0].strComment.empty());
    CHECK_EQ(vpwtx[0]->nOrderPos, (int64_t)1);
    CHECK_EQ(results[2].nTime, (int64_t)1333333336);
    CHECK_EQ(results[2].strOtherAccount, std::string("c"));

    ae.nTime = 1333333330;
    ae.strOtherAccount = "d";
    ae.nOrderPos = w.IncOrderPosNext();
    w.AddAccountingEntry(ae);

    GetResults(w, results);
    CHECK_EQ(results.size(), (size_t)3);
    CHECK_EQ(w.nOrderPosNext, (int64_t)4);
    CHECK_EQ(results[0].nTime, (int64_t)1333333333);
    CHECK_EQ(vpwtx[0]->nOrderPos, (int64_t)1);
    CHECK_EQ(results[2].nTime, (int64_t)1333333336);
    CHECK_EQ(results[3].nTime, (int64_t)1333333330);
    CHECK(results[3].strComment.empty());

    wtx.mapValue["comment"] = "y";
    Rehash(wtx);
    vpwtx.push_back(Add(w, wtx));
    vpwtx[1]->nTimeReceived = 1333333336;

    wtx.mapValue["comment"] = "x";
    Rehash(wtx);
    vpwtx.push_back(Add(w, wtx));
    vpwtx[2]->nTimeReceived = 1333333329;
    vpwtx[2]->nOrderPos = -1;

    GetResults(w, results);
    CHECK_EQ(results.size(), (size_t)3);
    CHECK_EQ(w.nOrderPosNext, (int64_t)6);
    CHECK_EQ(vpwtx[2]->nOrderPos, (int64_t)0);
    CHECK_EQ(results[1].nTime, (int64_t)1333333333);
    CHECK_EQ(vpwtx[0]->nOrderPos, (int64_t)2);
    CHECK_EQ(results[3].nTime, (int64_t)1333333336);
    CHECK_EQ(results[4].nTime, (int64_t)1333333330);
    CHECK(results[4].strComment.empty());
    CHECK_EQ(vpwtx[1]->nOrderPos, (int64_t)5);

    ae.nTime = 1333333334;
    ae.strOtherAccount = "e";
    ae.nOrderPos = -1;
    w.AddAccountingEntry(ae);

    GetResults(w, results);
    CHECK_EQ(results.size(), (size_t)4);
    CHECK_EQ(w.nOrderPosNext, (int64_t)7);
    CHECK_EQ(vpwtx[2]->nOrderPos, (int64_t)0);
    CHECK_EQ(results[1].nTime, (int64_t)1333333333);
    CHECK_EQ(vpwtx[0]->nOrderPos, (int64_t)2);
    CHECK_EQ(results[3].nTime, (int64_t)1333333336);
    CHECK(results[3].strComment.empty());
    CHECK_EQ(results[4].nTime, (int64_t)1333333330);
    CHECK(results[4].strComment.empty());
    CHECK_EQ(results[5].nTime, (int64_t)1333333334);
    CHECK_EQ(vpwtx[1]->nOrderPos, (int64_t)6);
}
