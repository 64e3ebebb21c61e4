// dos_tests: misbehaviour scoring, banning and the orphan pool limits.
// Parity: reference src/test/DoS_tests.cpp - DoS_banning (a peer at the ban threshold is banned
// at its next SendMessages, another address is not), DoS_banscore (-banscore moves the
// threshold), DoS_bantime (the ban lapses after -bantime), DoS_mapOrphans (orphans added with
// random parents, oversize orphans ignored, EraseOrphansFor a peer, LimitOrphanTxSize down to
// 40 / 10 / 0). Here additionally: whitelisted and local peers are never banned, and orphans
// expire after ORPHAN_TX_EXPIRE_TIME.
#include "test/unittest.h"

#include "net/net.h"
#include "net/net_processing.h"
#include "node/node.h"
#include "script/standard.h"
#include "util/util.h"

using namespace bcp;

namespace {

CAddress Ip(const char* ip) { return CAddress(LookupNumeric(std::string(ip) + ":8333", 8333), NODE_NONE); }

std::unique_ptr<CNode> Peer(NodeId id, const CAddress& addr, PeerLogicValidation& logic) {
    std::unique_ptr<CNode> n(new CNode(id, NODE_NETWORK, 0, -1, addr, 0, 0, "", true));
    n->SetSendVersion(PROTOCOL_VERSION);
    logic.InitializeNode(n.get());
    n->nVersion = 1;
    n->fSuccessfullyConnected = true;
    return n;
}

void Finish(PeerLogicValidation& logic, CNode& n) {
    bool dummy;
    logic.FinalizeNode(n.GetId(), dummy);
}

} // namespace

TEST_CASE(dos_tests, banning) {
    test::TestingSetup setup;
    CConnman connman(0x1337, 0x1337);
    PeerLogicValidation logic(&connman, setup.node->chainstate.get(), setup.node->mempool.get());
    std::atomic<bool> interrupt{false};
    const CAddress a1 = Ip("250.1.1.1"), a2 = Ip("250.1.1.2");
    auto n1 = Peer(0, a1, logic);
    logic.Misbehaving(n1->GetId(), 100); // the default threshold
    logic.SendMessages(n1.get(), interrupt);
    CHECK(connman.IsBanned(a1));
    CHECK(n1->fDisconnect);
    CHECK(!connman.IsBanned(Ip("250.1.1.3"))); // a different address
    // a second peer collects its score in steps
    auto n2 = Peer(1, a2, logic);
    logic.Misbehaving(n2->GetId(), 50);
    logic.SendMessages(n2.get(), interrupt);
    CHECK(!connman.IsBanned(a2));
    logic.Misbehaving(n2->GetId(), 50);
    logic.SendMessages(n2.get(), interrupt);
    CHECK(connman.IsBanned(a2));
    // whitelisted and local peers are disconnected, never banned
    auto w = Peer(2, Ip("250.1.1.4"), logic);
    w->fWhitelisted = true;
    logic.Misbehaving(w->GetId(), 100);
    logic.SendMessages(w.get(), interrupt);
    CHECK(!connman.IsBanned(Ip("250.1.1.4")));
    auto local = Peer(3, Ip("127.0.0.1"), logic);
    logic.Misbehaving(local->GetId(), 100);
    logic.SendMessages(local.get(), interrupt);
    CHECK(!connman.IsBanned(Ip("127.0.0.1")));
    CHECK(local->fDisconnect);
    for (CNode* n : {n1.get(), n2.get(), w.get(), local.get()}) Finish(logic, *n);
}

TEST_CASE(dos_tests, banscore) {
    test::TestingSetup setup;
    gArgs.ForceSetArg("-banscore", "111");
    CConnman connman(0x1337, 0x1337);
    PeerLogicValidation logic(&connman, setup.node->chainstate.get(), setup.node->mempool.get());
    std::atomic<bool> interrupt{false};
    const CAddress a1 = Ip("250.2.2.1");
    auto n1 = Peer(0, a1, logic);
    logic.Misbehaving(n1->GetId(), 100);
    logic.SendMessages(n1.get(), interrupt);
    CHECK(!connman.IsBanned(a1));
    logic.Misbehaving(n1->GetId(), 10);
    logic.SendMessages(n1.get(), interrupt);
    CHECK(!connman.IsBanned(a1));
    logic.Misbehaving(n1->GetId(), 1);
    logic.SendMessages(n1.get(), interrupt);
    CHECK(connman.IsBanned(a1));
    CNodeStateStats stats;
    REQUIRE(logic.GetNodeStateStats(n1->GetId(), stats));
    CHECK_EQ(stats.nMisbehavior, 111);
    gArgs.ClearArg("-banscore");
    Finish(logic, *n1);
}

TEST_CASE(dos_tests, bantime) {
    test::TestingSetup setup;
    const int64_t now = 1600000000;
    SetMockTime(now);
    CConnman connman(0x1337, 0x1337);
    PeerLogicValidation logic(&connman, setup.node->chainstate.get(), setup.node->mempool.get());
    std::atomic<bool> interrupt{false};
    const CAddress a = Ip("250.3.3.1");
    auto n = Peer(0, a, logic);
    logic.Misbehaving(n->GetId(), 100);
    logic.SendMessages(n.get(), interrupt);
    CHECK(connman.IsBanned(a));
    SetMockTime(now + 60 * 60);
    CHECK(connman.IsBanned(a));
    SetMockTime(now + DEFAULT_MISBEHAVING_BANTIME + 1);
    CHECK(!connman.IsBanned(a));
    SetMockTime(0);
    Finish(logic, *n);
}

TEST_CASE(dos_tests, orphans) {
    test::TestingSetup setup;
    CConnman connman(0x1337, 0x1337);
    PeerLogicValidation logic(&connman, setup.node->chainstate.get(), setup.node->mempool.get());
    FastRandomContext rng(true);
    CKey key;
    key.MakeNewKey(true);
    const CScript spk = GetScriptForDestination(key.GetPubKey().GetID());
    // 50 orphans spending random (unknown) parents
    std::vector<CTransactionRef> first;
    for (int i = 0; i < 50; i++) {
        CMutableTransaction tx;
        tx.vin.resize(1);
        tx.vin[0].prevout = COutPoint(rng.rand256(), 0);
        tx.vin[0].scriptSig << OP_1;
        tx.vout.resize(1);
        tx.vout[0].nValue = 1 * CENT;
        tx.vout[0].scriptPubKey = spk;
        first.push_back(MakeTransactionRef(tx));
        CHECK(logic.AddOrphanTx(first.back(), i));
    }
    // the same orphan twice is kept once
    CHECK(!logic.AddOrphanTx(first[0], 0));
    // 50 more spending the first ones
    for (int i = 0; i < 50; i++) {
        const CTransactionRef& parent = first[rng.randrange(first.size())];
        CMutableTransaction tx;
        tx.vin.resize(1);
        tx.vin[0].prevout = COutPoint(parent->GetHash(), 0);
        tx.vout.resize(1);
        tx.vout[0].nValue = (1 + i) * CENT; // distinct children of one parent
        tx.vout[0].scriptPubKey = spk;
        CHECK(logic.AddOrphanTx(MakeTransactionRef(tx), i));
    }
    CHECK_EQ(logic.OrphanCount(), 100u);
    // a large orphan (100 kB or more) is ignored
    {
        const CTransactionRef& parent = first[0];
        CMutableTransaction tx;
        tx.vout.resize(1);
        tx.vout[0].nValue = 1 * CENT;
        tx.vout[0].scriptPubKey = spk;
        tx.vin.resize(2777);
        for (size_t j = 0; j < tx.vin.size(); j++) tx.vin[j].prevout = COutPoint(parent->GetHash(), (uint32_t)j);
        CHECK(!logic.AddOrphanTx(MakeTransactionRef(tx), 0));
    }
    CHECK_EQ(logic.OrphanCount(), 100u);
    // everything from peers 0..2 goes when they disconnect
    for (NodeId p = 0; p < 3; p++) logic.EraseOrphansFor(p);
    CHECK_EQ(logic.OrphanCount(), 94u);
    // size limits
    logic.LimitOrphanTxSize(40);
    CHECK(logic.OrphanCount() <= 40u);
    logic.LimitOrphanTxSize(10);
    CHECK(logic.OrphanCount() <= 10u);
    logic.LimitOrphanTxSize(0);
    CHECK_EQ(logic.OrphanCount(), 0u);
    // expiry: orphans older than ORPHAN_TX_EXPIRE_TIME go at the next sweep
    const int64_t now = GetTime();
    SetMockTime(now);
    for (int i = 0; i < 5; i++) CHECK(logic.AddOrphanTx(first[i], 7));
    SetMockTime(now + 21 * 60);
    logic.LimitOrphanTxSize(100);
    CHECK_EQ(logic.OrphanCount(), 0u);
    SetMockTime(0);
}
