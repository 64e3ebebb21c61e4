// Block-index skip pointers, ancestors, locators, fork points and the time index.
// Parity: reference src/test/skiplist_tests.cpp (skiplist_test, getlocator_test,
// findearliestatleast_test). Here the index is a random tree of branches (not one side chain),
// and every query is checked against a plain walk over pprev.
#include "consensus/chain.h"
#include "test/unittest.h"

#include <deque>
#include <random>

namespace bcp {
namespace {

// A block tree: a main chain plus branches forking at random heights. Hashes encode
// (branch << 32 | height) so a locator entry tells where it came from.
struct Tree {
    std::deque<CBlockIndex> blocks; // stable addresses
    std::deque<uint256> hashes;
    CBlockIndex* Add(CBlockIndex* prev, uint32_t branch) {
        hashes.emplace_back();
        uint256& h = hashes.back();
        const uint64_t tag = ((uint64_t)branch << 32) | (uint32_t)(prev ? prev->nHeight + 1 : 0);
        memcpy(h.begin(), &tag, 8);
        blocks.emplace_back();
        CBlockIndex& b = blocks.back();
        b.pprev = prev;
        b.nHeight = prev ? prev->nHeight + 1 : 0;
        b.phashBlock = &h;
        b.BuildSkip();
        return &b;
    }
    static uint64_t Tag(const uint256& h) {
        uint64_t t;
        memcpy(&t, h.begin(), 8);
        return t;
    }
};

const CBlockIndex* WalkBack(const CBlockIndex* p, int height) {
    while (p && p->nHeight > height) p = p->pprev;
    return p;
}

} // namespace

TEST_CASE(skiplist_tests, ancestors_on_a_tree) {
    std::mt19937 rng(11);
    Tree t;
    std::vector<CBlockIndex*> main{t.Add(nullptr, 0)};
    for (int i = 1; i < 20000; i++) main.push_back(t.Add(main.back(), 0));
    std::vector<CBlockIndex*> tips{main.back()};
    for (uint32_t br = 1; br <= 30; br++) {
        CBlockIndex* p = main[rng() % main.size()];
        const int len = 1 + rng() % 3000;
        for (int i = 0; i < len; i++) p = t.Add(p, br);
        tips.push_back(p);
    }
    for (const CBlockIndex& b : t.blocks) {
        if (b.nHeight == 0) {
            CHECK(b.pskip == nullptr);
        } else {
            REQUIRE(b.pskip != nullptr);
            CHECK(b.pskip->nHeight < b.nHeight);
            CHECK(WalkBack(&b, b.pskip->nHeight) == b.pskip); // a real ancestor
        }
    }
    for (int q = 0; q < 3000; q++) {
        const CBlockIndex* tip = tips[rng() % tips.size()];
        const int h = rng() % (tip->nHeight + 1);
        CHECK(tip->GetAncestor(h) == WalkBack(tip, h));
        CHECK(tip->GetAncestor(0) == main[0]);
        CHECK(tip->GetAncestor(tip->nHeight) == tip);
        CHECK(tip->GetAncestor(tip->nHeight + 1) == nullptr);
        CHECK(tip->GetAncestor(-1) == nullptr);
    }
}

TEST_CASE(skiplist_tests, locators_and_forks) {
    std::mt19937 rng(5);
    Tree t;
    std::vector<CBlockIndex*> main{t.Add(nullptr, 0)};
    for (int i = 1; i < 50000; i++) main.push_back(t.Add(main.back(), 0));
    std::vector<CBlockIndex*> side;
    CBlockIndex* p = main[31415];
    for (int i = 0; i < 25000; i++) side.push_back(p = t.Add(p, 1));
    CChain chain;
    chain.SetTip(main.back());
    CHECK_EQ(chain.Height(), 49999);
    for (int q = 0; q < 200; q++) {
        const bool onSide = rng() & 1;
        const CBlockIndex* tip = onSide ? side[rng() % side.size()] : main[rng() % main.size()];
        CBlockLocator loc = chain.GetLocator(tip);
        REQUIRE(!loc.vHave.empty());
        CHECK(loc.vHave.front() == tip->GetBlockHash());
        CHECK(loc.vHave.back() == main[0]->GetBlockHash());
        // heights: the first eleven entries after the tip step back one block each, then the step
        // doubles; every entry is an ancestor of the tip
        int64_t prevH = tip->nHeight, step = 1;
        for (size_t i = 1; i + 1 < loc.vHave.size(); i++) {
            const uint64_t tag = Tree::Tag(loc.vHave[i]);
            const int64_t h = (int64_t)(uint32_t)tag;
            if (i > 11) step *= 2; // eleven single steps, then doubling
            CHECK_EQ(prevH - h, step);
            CHECK(WalkBack(tip, (int)h)->GetBlockHash() == loc.vHave[i]);
            prevH = h;
        }
        // the fork point of a side block with the main chain is the branch point
        const CBlockIndex* fork = chain.FindFork(tip);
        CHECK(fork == (onSide ? main[31415] : tip));
    }
    // the chain view: Contains / Next / operator[]
    CHECK(chain.Contains(main[100]));
    CHECK(!chain.Contains(side[0]));
    CHECK(chain.Next(main[100]) == main[101]);
    CHECK(chain.Next(main.back()) == nullptr);
    CHECK(chain[50000] == nullptr);
    // moving the tip to the side branch rewires the view
    chain.SetTip(side.back());
    CHECK(chain.Contains(side[5]));
    CHECK(!chain.Contains(main[40000]));
    CHECK(chain[31415] == main[31415]);
    CHECK(chain.FindFork(main[40000]) == main[31415]);
}

TEST_CASE(skiplist_tests, find_earliest_at_least) {
    std::mt19937 rng(99);
    Tree t;
    std::vector<CBlockIndex*> main{t.Add(nullptr, 0)};
    for (int i = 1; i < 60000; i++) main.push_back(t.Add(main.back(), 0));
    // block times wander (not monotone); nTimeMax is the running maximum
    unsigned int runmax = 0;
    int64_t clock = 1000000;
    for (CBlockIndex* b : main) {
        clock += (int64_t)(rng() % 1200) - 400;
        b->nTime = (unsigned int)clock;
        runmax = std::max(runmax, b->nTime);
        b->nTimeMax = runmax;
    }
    CChain chain;
    chain.SetTip(main.back());
    for (int q = 0; q < 5000; q++) {
        const int64_t when = main[rng() % main.size()]->nTime + (int64_t)(rng() % 5) - 2;
        const CBlockIndex* got = chain.FindEarliestAtLeast(when);
        // the first block whose running-maximum time reaches `when`, by linear scan
        const CBlockIndex* want = nullptr;
        for (CBlockIndex* b : main)
            if ((int64_t)b->nTimeMax >= when) {
                want = b;
                break;
            }
        CHECK(got == want);
    }
    CHECK(chain.FindEarliestAtLeast((int64_t)runmax + 1) == nullptr);
    CHECK(chain.FindEarliestAtLeast(0) == main[0]);
}

} // namespace bcp
