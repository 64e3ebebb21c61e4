// mempool_tests: CTxMemPool graph bookkeeping, orderings, eviction and the rolling minimum fee.
// Parity: reference src/test/mempool_tests.cpp (MempoolRemoveTest: recursive removal of a
// parent/child/grandchild tree; MempoolIndexingTest / MempoolAncestorIndexingTest: the
// descendant-score and ancestor-score orders; MempoolSizeLimitTest: TrimToSize evicts the lowest
// descendant-score packages, GetMinFee follows the removed package rate and halves per half-life
// once a block arrives; removeForBlock conflicts).
//
// The reference lists hand-computed orders for a dozen transactions; here every state is checked
// against a brute-force recomputation over the transaction graph (ancestor/descendant sets,
// aggregate sizes and modified fees, sort keys), on randomized DAGs, and TrimToSize is checked
// against a second pool driven by a naive "scan for the worst package" eviction.
#include "test/unittest.h"

#include "node/coins.h"
#include "node/policy.h"
#include "node/txmempool.h"
#include "util/util.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <set>

using namespace bcp;

namespace {

// A transaction spending `ins`, with `nOut` outputs; `salt` makes it unique and `pad` varies size.
CTransactionRef MakeTx(const std::vector<COutPoint>& ins, int nOut, uint32_t salt, int pad = 0) {
    CMutableTransaction m;
    for (const COutPoint& o : ins) {
        CScript sig;
        sig << std::vector<unsigned char>(4 + pad, (unsigned char)salt) << (int64_t)salt;
        m.vin.push_back(CTxIn(o, sig));
    }
    for (int i = 0; i < nOut; i++) m.vout.push_back(CTxOut(10000, CScript() << OP_TRUE));
    return MakeTransactionRef(std::move(m));
}

CTxMemPoolEntry Entry(const CTransactionRef& tx, Amount fee, int64_t time = 0, unsigned height = 1) {
    return CTxMemPoolEntry(tx, fee, time, 0.0, height, 0, false, 1, LockPoints());
}

COutPoint External(uint32_t i) {
    uint256 h;
    h.begin()[0] = 0xee;
    h.begin()[1] = (unsigned char)(i & 0xff);
    h.begin()[2] = (unsigned char)(i >> 8);
    h.begin()[3] = (unsigned char)(i >> 16);
    return COutPoint(h, 0);
}

// Brute-force view of the pool's graph, computed from the transactions alone.
struct Brute {
    std::map<uint256, CTransactionRef> txs;
    std::map<uint256, const CTxMemPoolEntry*> entry;
    explicit Brute(const CTxMemPool& pool) {
        for (const CTransactionRef& t : pool.AllTransactions()) {
            txs[t->GetHash()] = t;
            entry[t->GetHash()] = pool.GetEntry(t->GetHash());
        }
    }
    std::set<uint256> Parents(const uint256& h) const {
        std::set<uint256> r;
        for (const CTxIn& in : txs.at(h)->vin)
            if (txs.count(in.prevout.hash)) r.insert(in.prevout.hash);
        return r;
    }
    std::set<uint256> Ancestors(const uint256& h) const {
        std::set<uint256> r;
        std::vector<uint256> todo{h};
        while (!todo.empty()) {
            uint256 x = todo.back();
            todo.pop_back();
            for (const uint256& p : Parents(x))
                if (r.insert(p).second) todo.push_back(p);
        }
        return r;
    }
    std::set<uint256> Descendants(const uint256& h) const {
        std::set<uint256> r;
        for (const auto& kv : txs)
            if (kv.first != h && Ancestors(kv.first).count(h)) r.insert(kv.first);
        return r;
    }
    Amount ModFee(const uint256& h) const { return entry.at(h)->GetModifiedFee(); }
    uint64_t Size(const uint256& h) const { return entry.at(h)->GetTxSize(); }
};

// Every entry's ancestor/descendant aggregates equal a recomputation from the graph.
bool CheckAggregates(const CTxMemPool& pool, const char* where) {
    Brute b(pool);
    bool ok = true;
    uint64_t total = 0;
    for (const auto& kv : b.txs) {
        const uint256& h = kv.first;
        const CTxMemPoolEntry* e = b.entry.at(h);
        total += e->GetTxSize();
        const std::set<uint256> anc = b.Ancestors(h), desc = b.Descendants(h);
        uint64_t aSize = e->GetTxSize(), dSize = e->GetTxSize();
        Amount aFee = e->GetModifiedFee(), dFee = e->GetModifiedFee();
        for (const uint256& a : anc) aSize += b.Size(a), aFee += b.ModFee(a);
        for (const uint256& d : desc) dSize += b.Size(d), dFee += b.ModFee(d);
        if (e->GetCountWithAncestors() != anc.size() + 1 || e->GetSizeWithAncestors() != aSize ||
            e->GetModFeesWithAncestors() != aFee || e->GetCountWithDescendants() != desc.size() + 1 ||
            e->GetSizeWithDescendants() != dSize || e->GetModFeesWithDescendants() != dFee ||
            e->GetSigOpCountWithAncestors() != (int64_t)anc.size() + 1) {
            test::RecordFailure(std::string(where) + ": aggregates differ for " + h.ToString(), __FILE__, __LINE__);
            ok = false;
        }
        if (pool.GetAncestors(h).size() != anc.size() || pool.GetDescendants(h).size() != desc.size()) {
            test::RecordFailure(std::string(where) + ": ancestor/descendant query differs", __FILE__, __LINE__);
            ok = false;
        }
        for (const CTxIn& in : kv.second->vin) {
            if (pool.GetConflictTx(in.prevout) != kv.second.get()) {
                test::RecordFailure(std::string(where) + ": mapNextTx misses an input", __FILE__, __LINE__);
                ok = false;
            }
        }
    }
    if (pool.GetTotalTxSize() != total || pool.size() != b.txs.size()) {
        test::RecordFailure(std::string(where) + ": totals differ", __FILE__, __LINE__);
        ok = false;
    }
    return ok;
}

double OwnRate(const CTxMemPoolEntry* e) { return (double)e->GetModifiedFee() / e->GetTxSize(); }
double AncestorScoreOf(const CTxMemPoolEntry* e) {
    return std::min(OwnRate(e), (double)e->GetModFeesWithAncestors() / e->GetSizeWithAncestors());
}
double DescendantScoreOf(const CTxMemPoolEntry* e) {
    return std::max(OwnRate(e), (double)e->GetModFeesWithDescendants() / e->GetSizeWithDescendants());
}

// Builds a random DAG of `n` transactions; returns the outpoints that pool txs left unspent.
std::vector<COutPoint> FillRandom(CTxMemPool& pool, FastRandomContext& rng, int n, uint32_t saltBase,
                                  std::vector<COutPoint>& externalSpent, int64_t time0 = 0) {
    std::vector<COutPoint> unspent;
    uint32_t ext = saltBase * 4096;
    for (int i = 0; i < n; i++) {
        std::vector<COutPoint> ins;
        const int nIn = 1 + rng.randrange(3);
        for (int k = 0; k < nIn; k++) {
            if (!unspent.empty() && rng.randrange(4) != 0) {
                const size_t j = rng.randrange(unspent.size());
                ins.push_back(unspent[j]);
                unspent[j] = unspent.back();
                unspent.pop_back();
            } else {
                ins.push_back(External(ext++));
                externalSpent.push_back(ins.back());
            }
        }
        const int nOut = 1 + rng.randrange(3);
        CTransactionRef tx = MakeTx(ins, nOut, saltBase * 100000 + i, rng.randrange(120));
        pool.addUnchecked(tx->GetHash(), Entry(tx, 100 + rng.randrange(20000), time0 + i));
        for (int o = 0; o < nOut; o++) unspent.push_back(COutPoint(tx->GetHash(), o));
    }
    return unspent;
}

} // namespace

TEST_CASE(mempool_tests, remove_recursive) {
    test::BasicTestingSetup setup("regtest");
    CTxMemPool pool;
    // parent with 3 outputs -> 3 children -> 3 grandchildren
    CTransactionRef parent = MakeTx({External(1)}, 3, 1);
    std::vector<CTransactionRef> child, grand;
    for (int i = 0; i < 3; i++) {
        child.push_back(MakeTx({COutPoint(parent->GetHash(), i)}, 1, 10 + i));
        grand.push_back(MakeTx({COutPoint(child[i]->GetHash(), 0)}, 1, 20 + i));
    }
    // removing something absent is a no-op
    pool.removeRecursive(*parent);
    CHECK_EQ(pool.size(), 0u);
    pool.addUnchecked(parent->GetHash(), Entry(parent, 1000));
    pool.removeRecursive(*parent);
    CHECK_EQ(pool.size(), 0u);
    pool.addUnchecked(parent->GetHash(), Entry(parent, 1000));
    for (int i = 0; i < 3; i++) {
        pool.addUnchecked(child[i]->GetHash(), Entry(child[i], 1000));
        pool.addUnchecked(grand[i]->GetHash(), Entry(grand[i], 1000));
    }
    CheckAggregates(pool, "full tree");
    CHECK_EQ(pool.GetEntry(parent->GetHash())->GetCountWithDescendants(), 7u);
    // a child takes its grandchild with it
    pool.removeRecursive(*child[0]);
    CHECK_EQ(pool.size(), 5u);
    CheckAggregates(pool, "after child");
    // a grandchild alone
    pool.removeRecursive(*grand[1]);
    CHECK_EQ(pool.size(), 4u);
    CHECK_EQ(pool.GetEntry(parent->GetHash())->GetCountWithDescendants(), 4u);
    // the parent removes everything that is left
    pool.removeRecursive(*parent);
    CHECK_EQ(pool.size(), 0u);
    CHECK_EQ(pool.GetTotalTxSize(), 0u);
    CHECK(pool.mapNextTx.empty());
    // a tx whose parent is absent, removed by naming a tx that spends nothing of it: untouched
    pool.addUnchecked(child[2]->GetHash(), Entry(child[2], 1000));
    pool.removeRecursive(*grand[0]);
    CHECK_EQ(pool.size(), 1u);
    // removeRecursive of a tx that is not in the pool removes the in-pool spenders of its outputs
    pool.removeRecursive(*parent);
    CHECK_EQ(pool.size(), 0u);
}

TEST_CASE(mempool_tests, random_dag_aggregates) {
    test::BasicTestingSetup setup("regtest");
    FastRandomContext rng(true);
    for (int round = 0; round < 6; round++) {
        CTxMemPool pool;
        pool.setSanityCheck(1.0);
        std::vector<COutPoint> ext;
        FillRandom(pool, rng, 120, round + 1, ext);
        if (!CheckAggregates(pool, "after fill")) return;
        CCoinsView base;
        CCoinsViewCache view(&base);
        for (const COutPoint& o : ext) view.AddCoin(o, Coin(CTxOut(50000, CScript() << OP_TRUE), 1, false), false);
        pool.check(&view, 2); // throws on inconsistency

        for (int op = 0; op < 40 && pool.size() > 0; op++) {
            std::vector<CTransactionRef> all = pool.AllTransactions();
            const CTransactionRef pick = all[rng.randrange(all.size())];
            switch (rng.randrange(4)) {
            case 0: { // fee delta: must reach every ancestor's and descendant's aggregate
                pool.PrioritiseTransaction(pick->GetHash(), 0.0, (Amount)rng.randrange(5000) - 2500);
                break;
            }
            case 1: {
                pool.removeRecursive(*pick);
                break;
            }
            case 2: { // a block: `pick` plus its ancestors, and a conflicting spend of another tx's input
                Brute b(pool);
                std::set<uint256> blockSet = b.Ancestors(pick->GetHash());
                blockSet.insert(pick->GetHash());
                std::vector<CTransactionRef> vtx;
                // parents before children: sort by ancestor count
                std::vector<uint256> order(blockSet.begin(), blockSet.end());
                std::sort(order.begin(), order.end(), [&](const uint256& x, const uint256& y) {
                    return b.entry.at(x)->GetCountWithAncestors() < b.entry.at(y)->GetCountWithAncestors();
                });
                for (const uint256& h : order) vtx.push_back(b.txs.at(h));
                std::set<uint256> expectGone = blockSet;
                const CTransactionRef victim = all[rng.randrange(all.size())];
                if (!blockSet.count(victim->GetHash())) {
                    CTransactionRef conflict = MakeTx({victim->vin[0].prevout}, 1, 900000 + op);
                    vtx.push_back(conflict);
                    expectGone.insert(victim->GetHash());
                    for (const uint256& d : b.Descendants(victim->GetHash())) expectGone.insert(d);
                }
                const size_t before = pool.size();
                for (const CTransactionRef& t : vtx) AddCoins(view, *t, 2);
                pool.removeForBlock(vtx, 2);
                CHECK_EQ(pool.size(), before - expectGone.size());
                for (const uint256& h : expectGone) CHECK(!pool.exists(h));
                break;
            }
            case 3: { // expiry by entry time takes descendants along
                Brute b(pool);
                const int64_t cutoff = (int64_t)rng.randrange(120);
                std::set<uint256> expectGone;
                for (const auto& kv : b.entry)
                    if (kv.second->GetTime() < cutoff) {
                        expectGone.insert(kv.first);
                        for (const uint256& d : b.Descendants(kv.first)) expectGone.insert(d);
                    }
                const int removed = pool.Expire(cutoff);
                CHECK_EQ((size_t)removed, expectGone.size());
                break;
            }
            }
            if (!CheckAggregates(pool, "after op")) return;
        }
        pool.check(&view, 2);
    }
}

TEST_CASE(mempool_tests, orderings) {
    test::BasicTestingSetup setup("regtest");
    FastRandomContext rng(true);
    CTxMemPool pool;
    std::vector<COutPoint> ext;
    FillRandom(pool, rng, 200, 7, ext);
    // a few prioritisations so modified fees differ from base fees
    std::vector<CTransactionRef> all = pool.AllTransactions();
    for (int i = 0; i < 10; i++) pool.PrioritiseTransaction(all[rng.randrange(all.size())]->GetHash(), 0, 7000);

    // mining order: ancestor score (min of own and package rate) descending, then txid
    std::vector<CTxMemPool::txiter> mining = pool.SortedByAncestorScore();
    CHECK_EQ(mining.size(), pool.size());
    for (size_t i = 1; i < mining.size(); i++) {
        const double a = AncestorScoreOf(mining[i - 1]->second.get()), b = AncestorScoreOf(mining[i]->second.get());
        CHECK(a > b || (a == b && mining[i - 1]->first < mining[i]->first));
    }
    // relay order: depth first (a parent always precedes its children), then descendant score
    std::vector<CTransactionRef> relay = pool.AllTransactions();
    std::map<uint256, size_t> pos;
    for (size_t i = 0; i < relay.size(); i++) pos[relay[i]->GetHash()] = i;
    for (size_t i = 0; i < relay.size(); i++) {
        for (const CTxIn& in : relay[i]->vin)
            if (pos.count(in.prevout.hash)) CHECK(pos[in.prevout.hash] < i);
        if (i == 0) continue;
        const CTxMemPoolEntry* x = pool.GetEntry(relay[i - 1]->GetHash());
        const CTxMemPoolEntry* y = pool.GetEntry(relay[i]->GetHash());
        CHECK(x->GetCountWithAncestors() <= y->GetCountWithAncestors());
        if (x->GetCountWithAncestors() == y->GetCountWithAncestors())
            CHECK(DescendantScoreOf(x) >= DescendantScoreOf(y));
    }
    // infoAll follows the same order and reports the fee delta
    std::vector<TxMempoolInfo> info = pool.infoAll();
    REQUIRE(info.size() == relay.size());
    for (size_t i = 0; i < info.size(); i++) CHECK(info[i].tx->GetHash() == relay[i]->GetHash());
}

TEST_CASE(mempool_tests, ancestor_limits) {
    test::BasicTestingSetup setup("regtest");
    CTxMemPool pool;
    // a chain of 25: the 26th fails the ancestor-count limit, and the root's descendant limit
    std::vector<CTransactionRef> chain;
    COutPoint prev = External(77);
    for (int i = 0; i < 25; i++) {
        CTransactionRef t = MakeTx({prev}, 1, 3000 + i);
        pool.addUnchecked(t->GetHash(), Entry(t, 1000));
        chain.push_back(t);
        prev = COutPoint(t->GetHash(), 0);
    }
    CTransactionRef next = MakeTx({prev}, 1, 3999);
    CTxMemPoolEntry e = Entry(next, 1000);
    CTxMemPool::setEntries anc;
    std::string err;
    const uint64_t big = std::numeric_limits<uint64_t>::max();
    CHECK(!pool.CalculateMemPoolAncestors(e, anc, 25, big, big, big, err));
    CHECK(!err.empty());
    anc.clear();
    err.clear();
    CHECK(pool.CalculateMemPoolAncestors(e, anc, 26, big, big, big, err));
    CHECK_EQ(anc.size(), 25u);
    anc.clear();
    CHECK(!pool.CalculateMemPoolAncestors(e, anc, 26, big, 25, big, err)); // root would get 26 descendants
    anc.clear();
    // ancestor size limit in bytes (limits are in kB in policy, bytes here)
    const uint64_t chainSize = pool.GetEntry(chain.back()->GetHash())->GetSizeWithAncestors();
    CHECK(!pool.CalculateMemPoolAncestors(e, anc, big, chainSize, big, big, err));
    anc.clear();
    CHECK(pool.CalculateMemPoolAncestors(e, anc, big, chainSize + e.GetTxSize(), big, big, err));
}

TEST_CASE(mempool_tests, trim_to_size_matches_naive_eviction) {
    test::BasicTestingSetup setup("regtest");
    FastRandomContext rng(true);
    for (int round = 0; round < 4; round++) {
        CTxMemPool a, b;
        std::vector<COutPoint> ext;
        // identical contents in both pools (same seed)
        FastRandomContext r1(rng.rand256());
        FastRandomContext r2 = r1;
        FillRandom(a, r1, 400, 20 + round, ext);
        FillRandom(b, r2, 400, 20 + round, ext);
        REQUIRE(a.size() == b.size() && a.DynamicMemoryUsage() == b.DynamicMemoryUsage());
        const size_t limit = a.DynamicMemoryUsage() * (40 + 15 * round) / 100;

        a.TrimToSize(limit);
        CHECK(a.DynamicMemoryUsage() <= limit);
        // naive eviction: scan for the lowest descendant score (newest, then lowest txid on ties)
        double maxRemovedRate = 0;
        while (b.DynamicMemoryUsage() > limit) {
            const CTxMemPoolEntry* worst = nullptr;
            for (const CTransactionRef& t : b.AllTransactions()) {
                const CTxMemPoolEntry* e = b.GetEntry(t->GetHash());
                if (!worst) { worst = e; continue; }
                const double s = DescendantScoreOf(e), w = DescendantScoreOf(worst);
                if (s < w || (s == w && (e->GetTime() > worst->GetTime() ||
                                         (e->GetTime() == worst->GetTime() && e->GetTx().GetHash() < worst->GetTx().GetHash()))))
                    worst = e;
            }
            const double rate = (double)CFeeRate(worst->GetModFeesWithDescendants(), worst->GetSizeWithDescendants()).GetFeePerK() +
                                (double)incrementalRelayFee.GetFeePerK();
            maxRemovedRate = std::max(maxRemovedRate, rate);
            const CTransactionRef victim = worst->GetSharedTx();
            b.removeRecursive(*victim);
        }
        CHECK_EQ(a.size(), b.size());
        for (const CTransactionRef& t : b.AllTransactions()) CHECK(a.exists(t->GetHash()));
        CheckAggregates(a, "after trim");
        // no block since the bump: the minimum fee is exactly the highest removed package rate
        CHECK_EQ((double)a.GetMinFee(limit).GetFeePerK(), maxRemovedRate);
    }
}

TEST_CASE(mempool_tests, rolling_min_fee_decay) {
    test::BasicTestingSetup setup("regtest");
    const int64_t t0 = 1500000000;
    SetMockTime(t0);
    CTxMemPool pool;
    // one cheap and one expensive standalone tx; trim the cheap one out
    CTransactionRef cheap = MakeTx({External(500)}, 1, 500, 100);
    CTransactionRef dear = MakeTx({External(501)}, 1, 501, 100);
    pool.addUnchecked(cheap->GetHash(), Entry(cheap, 10000));
    pool.addUnchecked(dear->GetHash(), Entry(dear, 90000));
    const size_t big = pool.DynamicMemoryUsage();
    pool.TrimToSize(big - 1);
    CHECK(!pool.exists(cheap->GetHash()));
    CHECK(pool.exists(dear->GetHash()));
    const Amount bumped = CFeeRate(10000, cheap->GetTotalSize()).GetFeePerK() + incrementalRelayFee.GetFeePerK();
    // a size limit far above usage (usage < limit/4) quarters the half-life
    const size_t limit = big * 100;
    CHECK_EQ(pool.GetMinFee(limit).GetFeePerK(), bumped);
    // without a block nothing decays, however much time passes
    const int64_t halflife = 60 * 60 * 12 / 4;
    SetMockTime(t0 + halflife / 2);
    CHECK_EQ(pool.GetMinFee(limit).GetFeePerK(), bumped);
    // a block arrives: decay runs from the block's time, in steps of at least 10 s
    const int64_t tb = t0 + halflife / 2;
    pool.removeForBlock({}, 2);
    SetMockTime(tb + 5);
    CHECK_EQ(pool.GetMinFee(limit).GetFeePerK(), bumped);
    SetMockTime(tb + halflife);
    CHECK_EQ(pool.GetMinFee(limit).GetFeePerK(), std::max<Amount>(bumped / 2, incrementalRelayFee.GetFeePerK()));
    SetMockTime(tb + 2 * halflife);
    const double expected = (double)bumped / 4;
    const Amount got = pool.GetMinFee(limit).GetFeePerK();
    if (expected < (double)incrementalRelayFee.GetFeePerK() / 2) CHECK_EQ(got, 0);
    else CHECK_EQ(got, std::max<Amount>((Amount)expected, incrementalRelayFee.GetFeePerK()));
    // far in the future the floor drops to zero (below half the incremental fee)
    SetMockTime(tb + 40 * halflife);
    CHECK_EQ(pool.GetMinFee(limit).GetFeePerK(), 0);
    SetMockTime(0);
}
