// ConnectBlock's parallel UTXO pass against the serial one.
// Parity: the UTXO rules of reference src/validation.cpp ConnectBlock (:2011-2127: missing or
// spent inputs, BIP68, sigop limits, input values, coinbase maturity, AddCoins/SpendCoin, undo
// records) and CheckTxInputs (src/consensus/tx_verify.cpp). The reference has one serial pass;
// these cases pin that the parallel pass (taken for blocks of -parallelutxo transactions or more)
// leaves the same coins and undo data, and that a block it refuses gets the serial pass's exact
// reject reason.
#include "test/unittest.h"
#include "util/sync.h"

#include "consensus/merkle.h"
#include "node/miner.h"
#include "node/sigverify.h"
#include "node/txdb.h"
#include "node/validation.h"
#include "script/sign.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <cstdio>
#include <cstring>
#include <map>
#include <random>

using namespace bcp;

namespace {

CScript P2PK(const CKey& k) { return CScript() << k.GetPubKey().Raw() << OP_CHECKSIG; }

struct Prev {
    CTransaction tx;
    uint32_t n;
};

// spend `ins` (all P2PK to `key`) into `outs`
CMutableTransaction Make(const std::vector<Prev>& ins, const std::vector<CTxOut>& outs, const CKey& key) {
    CMutableTransaction m;
    for (const Prev& p : ins) m.vin.push_back(CTxIn(COutPoint(p.tx.GetHash(), p.n), CScript()));
    m.vout = outs;
    CBasicKeyStore ks;
    ks.AddKey(key);
    for (size_t i = 0; i < ins.size(); i++) {
        const CTxOut& o = ins[i].tx.vout[ins[i].n];
        if (o.scriptPubKey.IsUnspendable()) continue; // refused before its script runs
        if (!SignSignature(ks, o.scriptPubKey, m, (unsigned)i, o.nValue, SIGHASH_ALL | SIGHASH_FORKID))
            throw std::runtime_error("test: signing failed");
    }
    return m;
}

// every coin the block touches, as the tip's view now has it ("" = none)
std::map<std::string, std::string> Snapshot(Chainstate& cs, const std::vector<CMutableTransaction>& txs,
                                            const std::vector<COutPoint>& extra) {
    std::map<std::string, std::string> out;
    auto add = [&](const COutPoint& op) {
        Coin c;
        std::string v;
        if (cs.CoinsTip().GetCoin(op, c) && !c.IsSpent())
            v = strprintf("%lld/%u/%d/%s", (long long)c.out.nValue, c.nHeight, (int)c.fCoinBase,
                          HexStr(c.out.scriptPubKey).c_str());
        out[op.ToString()] = v;
    };
    for (const CMutableTransaction& m : txs) {
        const CTransaction t(m);
        for (const CTxIn& in : t.vin) add(in.prevout);
        for (size_t o = 0; o < t.vout.size(); o++) add(COutPoint(t.GetHash(), (uint32_t)o));
    }
    for (const COutPoint& op : extra) add(op);
    return out;
}

CBlock Assemble(Chainstate& cs, const std::vector<CMutableTransaction>& txs, const CScript& spk) {
    BlockAssembler ba(cs, nullptr);
    std::unique_ptr<CBlockTemplate> t = ba.CreateNewBlock(spk);
    CBlock b = t->block;
    b.vtx.resize(1);
    for (const CMutableTransaction& m : txs) b.vtx.push_back(MakeTransactionRef(m));
    unsigned extra = 0;
    IncrementExtraNonce(&b, cs.TipNow(), extra, cs.MaxBlockSize());
    return b;
}

// TestBlockValidity's reject reason with the parallel pass forced on (1) and off (0)
std::pair<std::string, std::string> Verdicts(Chainstate& cs, const CBlock& b) {
    std::string r[2];
    for (int par = 0; par < 2; par++) {
        cs.SetParallelUtxoMinTx(par ? 1 : 0);
        CValidationState st;
        r[par] = cs.TestBlockValidity(st, b, cs.TipNow(), false, true) ? "valid" : st.GetRejectReason();
    }
    cs.SetParallelUtxoMinTx(64);
    return {r[0], r[1]};
}

bool Same(const std::map<std::string, std::string>& a, const std::map<std::string, std::string>& b) {
    for (const auto& kv : a)
        if (!b.count(kv.first) || b.at(kv.first) != kv.second)
            std::printf("  %s: '%s' vs '%s'\n", kv.first.c_str(), kv.second.c_str(),
                        b.count(kv.first) ? b.at(kv.first).c_str() : "(absent)");
    return a == b;
}

} // namespace

TEST_CASE(connectblock_tests, parallel_pass_matches_serial) {
    test::TestChain100Setup setup;
    Chainstate& cs = *setup.node->chainstate;
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    for (int i = 0; i < 10; i++) setup.CreateAndProcessBlock({}, spk);
    // a fan-out, 70 children of it (two outputs each, every fifth with an OP_RETURN too), 35
    // grandchildren spending a child's first output, and 6 spends of mature coinbases
    std::vector<CMutableTransaction> txs;
    const Amount fanEach = (setup.coinbaseTxns[0].vout[0].nValue - 100000) / 70;
    txs.push_back(Make({{setup.coinbaseTxns[0], 0}}, std::vector<CTxOut>(70, CTxOut(fanEach, spk)), key));
    const CTransaction fan(txs[0]);
    std::vector<CTransaction> children;
    for (uint32_t i = 0; i < 70; i++) {
        std::vector<CTxOut> outs{CTxOut(fanEach / 2 - 1000, spk), CTxOut(fanEach / 2 - 1000, spk)};
        if (i % 5 == 0) outs.push_back(CTxOut(0, CScript() << OP_RETURN << std::vector<unsigned char>(4, (unsigned char)i)));
        txs.push_back(Make({{fan, i}}, outs, key));
        children.emplace_back(txs.back());
    }
    for (uint32_t i = 0; i < 35; i++)
        txs.push_back(Make({{children[2 * i], 0}}, {CTxOut(fanEach / 2 - 5000, spk)}, key));
    for (int c = 1; c <= 6; c++)
        txs.push_back(Make({{setup.coinbaseTxns[c], 0}}, {CTxOut(setup.coinbaseTxns[c].vout[0].nValue - 2000, spk)}, key));
    REQUIRE(txs.size() >= 64);
    const std::vector<COutPoint> none;
    const auto before = Snapshot(cs, txs, none);

    // both passes accept it
    const CBlock probe = Assemble(cs, txs, spk);
    const auto v = Verdicts(cs, probe);
    CHECK_EQ(v.first, std::string("valid"));
    CHECK_EQ(v.second, std::string("valid"));

    // connect it with the parallel pass (the default threshold; the block has 112 transactions)
    const int64_t fastBefore = cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO);
    const CBlock blk = setup.CreateAndProcessBlock(txs, spk);
    CHECK_EQ(cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO), fastBefore + 1);
    const COutPoint cbOut(blk.vtx[0]->GetHash(), 0);
    const auto parallel = Snapshot(cs, txs, {cbOut});
    // what it must hold: every input spent; outputs spent inside the block and OP_RETURNs absent;
    // the rest at the block's height, the coinbase flagged
    const int h = cs.HeightNow();
    for (const CMutableTransaction& m : txs)
        for (const CTxIn& in : m.vin) CHECK_EQ(parallel.at(in.prevout.ToString()), std::string());
    for (uint32_t i = 0; i < 70; i++) {
        const std::string first = parallel.at(COutPoint(children[i].GetHash(), 0).ToString());
        CHECK_EQ(first.empty(), i % 2 == 0);
        CHECK(!parallel.at(COutPoint(children[i].GetHash(), 1).ToString()).empty());
        if (i % 5 == 0) CHECK(parallel.at(COutPoint(children[i].GetHash(), 2).ToString()).empty());
    }
    const std::string cb = parallel.at(cbOut.ToString());
    CHECK(cb.find(strprintf("/%d/1/", h)) != std::string::npos);
    const std::string last = parallel.at(COutPoint(CTransaction(txs.back()).GetHash(), 0).ToString());
    CHECK(last.find(strprintf("/%d/0/", h)) != std::string::npos);
    {
        // the in-place update leaves no tip entry at all for an output created and spent inside
        // the block (as AddCoin + SpendCoin of a FRESH entry would not)
        std::lock_guard<CCriticalSection> l(cs.cs());
        for (uint32_t i = 0; i < 35; i++) CHECK(cs.CoinsTip().FindInCache(COutPoint(children[2 * i].GetHash(), 0)) == nullptr);
    }

    // disconnecting with the parallel pass's undo data restores every spent coin exactly
    CBlockIndex* pindex = cs.LookupBlockIndex(blk.GetHash());
    REQUIRE(pindex != nullptr);
    CValidationState st;
    REQUIRE(cs.InvalidateBlock(st, pindex));
    CHECK(Same(before, Snapshot(cs, txs, none)));

    // and the serial pass, reconnecting the same block, leaves the same coins
    cs.SetParallelUtxoMinTx(0);
    REQUIRE(cs.ResetBlockFailureFlags(pindex));
    REQUIRE(cs.ActivateBestChain(st));
    REQUIRE(cs.TipNow() == pindex);
    CHECK(Same(parallel, Snapshot(cs, txs, {cbOut})));
    cs.SetParallelUtxoMinTx(64);
}

TEST_CASE(connectblock_tests, parallel_pass_reject_reasons) {
    test::TestChain100Setup setup;
    Chainstate& cs = *setup.node->chainstate;
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    for (int i = 0; i < 5; i++) setup.CreateAndProcessBlock({}, spk);
    const Amount v0 = setup.coinbaseTxns[0].vout[0].nValue;
    const CMutableTransaction fan = Make({{setup.coinbaseTxns[0], 0}},
                                         {CTxOut(v0 / 4, spk), CTxOut(v0 / 4, spk),
                                          CTxOut(0, CScript() << OP_RETURN), CTxOut(v0 / 4, spk)},
                                         key);
    const CTransaction f(fan);
    auto spend = [&](const CTransaction& p, uint32_t n, Amount v) { return Make({{p, n}}, {CTxOut(v, spk)}, key); };
    const Amount small = v0 / 8;
    struct Case {
        const char* what;
        std::vector<CMutableTransaction> txs;
    };
    const CTransaction cbImmature = setup.coinbaseTxns.back();
    CMutableTransaction beyond = spend(f, 0, small);
    beyond.vin[0].prevout.n = 9; // no such output (signature no longer matters: the input is missing)
    std::vector<Case> cases{
        {"in-block output spent twice", {fan, spend(f, 0, small), spend(f, 0, small / 2)}},
        {"tip coin spent twice", {spend(setup.coinbaseTxns[1], 0, small), spend(setup.coinbaseTxns[1], 0, small / 2)}},
        {"child before its parent", {spend(f, 1, small), fan}},
        {"missing output of an in-block tx", {fan, beyond}},
        {"in-block OP_RETURN output spent", {fan, spend(f, 2, 0)}},
        {"outputs above inputs", {fan, spend(f, 3, v0)}},
        {"immature coinbase", {spend(cbImmature, 0, small)}},
        {"valid chain", {fan, spend(f, 0, small), spend(f, 1, small), spend(f, 3, small)}},
    };
    for (const Case& c : cases) {
        const CBlock b = Assemble(cs, c.txs, spk);
        const auto v = Verdicts(cs, b);
        if (v.second != v.first) std::printf("  %s: serial %s, parallel %s\n", c.what, v.first.c_str(), v.second.c_str());
        CHECK_EQ(v.second, v.first);
        if (std::string(c.what) == "valid chain") CHECK_EQ(v.first, std::string("valid"));
        else CHECK(v.first != "valid");
    }
}

// DecodeBlock (the parallel decode of blocks read for connecting) against the stream decode.
TEST_CASE(blockdecode_tests, parallel_decode_matches_stream) {
    std::mt19937_64 rng(7);
    CBlock b;
    b.nVersion = 4;
    b.nHeight = 5000;
    b.nBits = 0x207fffff;
    for (int i = 0; i < 700; i++) {
        CMutableTransaction m;
        m.nVersion = 1 + (int)(rng() % 2);
        m.nLockTime = (uint32_t)rng();
        const int nin = 1 + (int)(rng() % 4), nout = 1 + (int)(rng() % 5);
        for (int k = 0; k < nin; k++) {
            uint256 h;
            for (int w = 0; w < 4; w++) {
                const uint64_t x = rng();
                memcpy(h.begin() + 8 * w, &x, 8);
            }
            m.vin.push_back(CTxIn(COutPoint(h, (uint32_t)(rng() % 7)),
                                  CScript(std::vector<unsigned char>(rng() % 300, (unsigned char)k)), (uint32_t)rng()));
        }
        for (int k = 0; k < nout; k++)
            m.vout.push_back(CTxOut((Amount)(rng() % 100000000), CScript(std::vector<unsigned char>(rng() % 60, 0x51))));
        b.vtx.push_back(MakeTransactionRef(std::move(m)));
    }
    DataStream s(SER_DISK, PROTOCOL_VERSION);
    s << b;
    const std::vector<unsigned char> raw((const unsigned char*)s.data(), (const unsigned char*)s.data() + s.size());
    WorkerPool pool(4);
    for (WorkerPool* p : {(WorkerPool*)nullptr, &pool}) {
        CBlock got;
        REQUIRE(DecodeBlock(raw.data(), raw.size(), got, p));
        CHECK(got.GetBlockHeader().GetHash() == b.GetBlockHeader().GetHash());
        REQUIRE(got.vtx.size() == b.vtx.size());
        bool same = true;
        for (size_t i = 0; i < b.vtx.size(); i++) same &= got.vtx[i]->GetHash() == b.vtx[i]->GetHash();
        CHECK(same);
    }
    // the block size from the transactions' cached sizes matches a full serialization walk, in
    // both header formats
    for (int v : {PROTOCOL_VERSION, PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY})
        CHECK_EQ(BlockSerializeSize(b, v), (uint64_t)GetSerializeSize(b, v));
    CHECK_EQ(b.vtx[5]->GetTotalSize(), (unsigned)GetSerializeSize(*b.vtx[5], PROTOCOL_VERSION));
    // a block cut anywhere fails both ways, like the stream decode
    for (int t = 0; t < 40; t++) {
        const size_t cut = 81 + rng() % (raw.size() - 82);
        CBlock a, c;
        DataStream ss((const char*)raw.data(), (const char*)raw.data() + cut, SER_DISK, PROTOCOL_VERSION);
        bool streamOk = true;
        try {
            ss >> a;
        } catch (const std::exception&) {
            streamOk = false;
        }
        CHECK(!streamOk);
        CHECK(!DecodeBlock(raw.data(), cut, c, &pool));
        CHECK(c.vtx.empty());
    }
    // an absurd transaction count is refused before anything is allocated for it
    std::vector<unsigned char> bogus(raw.begin(), raw.begin() + 200);
    SpanReader hr(raw.data(), raw.size(), SER_DISK, PROTOCOL_VERSION);
    CBlockHeader h;
    h.Unserialize(hr);
    const size_t hdrLen = hr.tell();
    bogus.resize(hdrLen);
    bogus.push_back(0xfe);
    for (unsigned char x : {0xff, 0xff, 0xff, 0x01}) bogus.push_back(x);
    CBlock d;
    CHECK(!DecodeBlock(bogus.data(), bogus.size(), d, &pool));
}

TEST_CASE(connectblock_tests, parallel_pass_with_bip34_active) {
    // Mainnet and testnet stop enforcing BIP30 once the BIP34 block is buried (every mainnet
    // block above 227931). The parallel UTXO pass must still run there: activate BIP34 on this
    // regtest chain at height 5 (its hash pinned), connect a 64+ transaction block, and check
    // that the parallel pass took it and agrees with the serial pass.
    test::TestChain100Setup setup;
    Chainstate& cs = *setup.node->chainstate;
    Consensus::Params& cons = const_cast<CChainParams&>(Params()).MutableConsensus();
    const int savedHeight = cons.BIP34Height;
    const uint256 savedHash = cons.BIP34Hash;
    cons.BIP34Height = 5;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        cons.BIP34Hash = cs.ActiveChain()[5]->GetBlockHash();
    }
    struct Restore {
        Consensus::Params& c;
        int h;
        uint256 hh;
        ~Restore() {
            c.BIP34Height = h;
            c.BIP34Hash = hh;
        }
    } restore{cons, savedHeight, savedHash};
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    for (int i = 0; i < 3; i++) setup.CreateAndProcessBlock({}, spk);
    std::vector<CMutableTransaction> txs;
    const Amount each = (setup.coinbaseTxns[0].vout[0].nValue - 100000) / 80;
    txs.push_back(Make({{setup.coinbaseTxns[0], 0}}, std::vector<CTxOut>(80, CTxOut(each, spk)), key));
    const CTransaction fan(txs[0]);
    for (uint32_t i = 0; i < 70; i++) txs.push_back(Make({{fan, i}}, {CTxOut(each - 1000, spk)}, key));
    const auto v = Verdicts(cs, Assemble(cs, txs, spk));
    CHECK_EQ(v.first, std::string("valid"));
    CHECK_EQ(v.second, std::string("valid"));
    const int64_t fastBefore = cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO);
    const CBlock blk = setup.CreateAndProcessBlock(txs, spk);
    CHECK_EQ(cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO), fastBefore + 1);
    std::lock_guard<CCriticalSection> l(cs.cs());
    CHECK(cs.Tip()->GetBlockHash() == blk.GetHash());
}

// ConnectTip lets the parallel UTXO pass update the coins tip in place (no per-block view to
// merge). A block that fails after that update (here: its coinbase claims more than subsidy plus
// fees, checked after the UTXO pass) must leave the tip exactly as it was, and the chain then
// connects the honest version of the same block through the same path.
TEST_CASE(connectblock_tests, in_place_tip_update_undone_on_failure) {
    test::TestChain100Setup setup;
    Chainstate& cs = *setup.node->chainstate;
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    for (int i = 0; i < 3; i++) setup.CreateAndProcessBlock({}, spk);
    std::vector<CMutableTransaction> txs;
    const Amount each = (setup.coinbaseTxns[0].vout[0].nValue - 100000) / 80;
    txs.push_back(Make({{setup.coinbaseTxns[0], 0}}, std::vector<CTxOut>(80, CTxOut(each, spk)), key));
    const CTransaction fan(txs[0]);
    for (uint32_t i = 0; i < 70; i++) txs.push_back(Make({{fan, i}}, {CTxOut(each - 1000, spk)}, key));
    for (int c = 1; c <= 2; c++) // mature coinbases (heights 2 and 3; the block is at 104)
        txs.push_back(Make({{setup.coinbaseTxns[c], 0}}, {CTxOut(setup.coinbaseTxns[c].vout[0].nValue - 2000, spk)}, key));
    const std::vector<COutPoint> none;
    std::map<std::string, std::string> before;
    uint256 tipBefore;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        before = Snapshot(cs, txs, none);
        tipBefore = cs.Tip()->GetBlockHash();
    }
    CBlock greedy = Assemble(cs, txs, spk);
    CMutableTransaction cb(*greedy.vtx[0]);
    cb.vout[0].nValue += 50 * COIN;
    greedy.vtx[0] = MakeTransactionRef(cb);
    greedy.hashMerkleRoot = BlockMerkleRoot(greedy);
    uint64_t tries = 1u << 30;
    REQUIRE(SolveBlock(greedy, Params(), tries, false));
    const int64_t fast0 = cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO);
    bool fNew = false;
    CValidationState st;
    cs.ProcessNewBlock(std::make_shared<const CBlock>(greedy), true, &fNew, &st);
    CHECK_EQ(cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO), fast0 + 1); // it got to the in-place update
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        CHECK(cs.Tip()->GetBlockHash() == tipBefore);
        CHECK(Same(before, Snapshot(cs, txs, none)));
        CHECK_EQ(Snapshot(cs, {}, {COutPoint(greedy.vtx[0]->GetHash(), 0)}).begin()->second, std::string());
        CHECK(cs.CoinsTip().GetBestBlock() == tipBefore);
    }
    const CBlock honest = setup.CreateAndProcessBlock(txs, spk);
    CHECK_EQ(cs.ConnectPhaseMicros(Chainstate::PH_FASTUTXO), fast0 + 2);
    std::lock_guard<CCriticalSection> l(cs.cs());
    CHECK(cs.Tip()->GetBlockHash() == honest.GetHash());
    const auto after = Snapshot(cs, txs, none);
    for (const CMutableTransaction& m : txs)
        for (const CTxIn& in : m.vin) CHECK_EQ(after.at(in.prevout.ToString()), std::string());
}

// After the BIP34 block BIP30 is no longer checked, so a coinbase whose first output is already
// an unspent coin replaces it (AddCoins with possible_overwrite, reference src/coins.cpp:97-134 and
// src/validation.cpp:1952-1990). The same post-BIP34 block is connected by two fresh chainstates,
// one through the parallel UTXO pass and one through the serial pass: the verdicts, the coins the
// block touches (the overwritten coin included) and the undo bytes on disk are identical, and a
// variant that double-spends gets the same reject reason from both.
TEST_CASE(connectblock_tests, post_bip34_coinbase_overwrite_both_paths) {
    test::TestChain100Setup setup;
    Chainstate& a = *setup.node->chainstate;
    Consensus::Params& cons = const_cast<CChainParams&>(Params()).MutableConsensus();
    const int savedHeight = cons.BIP34Height;
    const uint256 savedHash = cons.BIP34Hash;
    cons.BIP34Height = 5;
    {
        std::lock_guard<CCriticalSection> l(a.cs());
        cons.BIP34Hash = a.ActiveChain()[5]->GetBlockHash();
    }
    struct Restore {
        Consensus::Params& c;
        int h;
        uint256 hh;
        ~Restore() {
            c.BIP34Height = h;
            c.BIP34Hash = hh;
        }
    } restore{cons, savedHeight, savedHash};
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    for (int i = 0; i < 3; i++) setup.CreateAndProcessBlock({}, spk);
    std::vector<std::shared_ptr<const CBlock>> chain; // a's blocks above genesis, in height order
    for (const CBlockIndex* p = a.TipNow(); p && p->pprev; p = p->pprev) {
        auto b = std::make_shared<CBlock>();
        REQUIRE(ReadBlockFromDisk(*b, p, Params(), true));
        chain.insert(chain.begin(), b);
    }
    std::vector<CMutableTransaction> txs;
    const Amount each = (setup.coinbaseTxns[0].vout[0].nValue - 100000) / 80;
    txs.push_back(Make({{setup.coinbaseTxns[0], 0}}, std::vector<CTxOut>(80, CTxOut(each, spk)), key));
    const CTransaction fan(txs[0]);
    for (uint32_t i = 0; i < 70; i++) txs.push_back(Make({{fan, i}}, {CTxOut(each - 1000, spk)}, key));
    CBlock blk = Assemble(a, txs, spk);
    uint64_t tries = 1u << 30;
    REQUIRE(SolveBlock(blk, Params(), tries, false));
    const COutPoint cbOut(blk.vtx[0]->GetHash(), 0);
    // the double-spending variant: one more transaction spending fan output 0 again
    std::vector<CMutableTransaction> bad = txs;
    bad.push_back(Make({{fan, 0}}, {CTxOut(each - 2000, spk)}, key));
    const CBlock badBlk = Assemble(a, bad, spk);

    struct Result {
        std::pair<std::string, std::string> verdict, badVerdict;
        std::map<std::string, std::string> coins;
        std::vector<unsigned char> undo;
        int64_t fast = 0;
    } res[2];
    for (int par = 0; par < 2; par++) {
        ChainstateOptions o;
        o.memoryOnly = true;
        char tmpl[] = "/tmp/bcp_test_bip34ow_XXXXXX";
        REQUIRE(mkdtemp(tmpl) != nullptr);
        o.datadir = tmpl;
        o.useGpu = false;
        Chainstate b(Params(), o);
        std::string err;
        REQUIRE(b.InitBlockIndex(err));
        for (const auto& c : chain) {
            bool fNew = false;
            CValidationState st;
            REQUIRE(b.ProcessNewBlock(c, true, &fNew, &st));
        }
        REQUIRE(b.TipNow()->GetBlockHash() == a.TipNow()->GetBlockHash());
        {
            // an earlier coinbase with this txid whose first output is still unspent
            std::lock_guard<CCriticalSection> l(b.cs());
            b.CoinsTip().AddCoin(cbOut, Coin(CTxOut(12345, spk), 7, true), true);
        }
        Result& r = res[par];
        r.verdict = Verdicts(b, blk);
        r.badVerdict = Verdicts(b, badBlk);
        b.SetParallelUtxoMinTx(par ? 1 : 0);
        const int64_t fast0 = b.ConnectPhaseMicros(Chainstate::PH_FASTUTXO);
        bool fNew = false;
        CValidationState st;
        REQUIRE(b.ProcessNewBlock(std::make_shared<const CBlock>(blk), true, &fNew, &st));
        r.fast = b.ConnectPhaseMicros(Chainstate::PH_FASTUTXO) - fast0;
        {
            std::lock_guard<CCriticalSection> l(b.cs());
            CHECK(b.Tip()->GetBlockHash() == blk.GetHash());
            r.coins = Snapshot(b, txs, {cbOut});
            const CBlockIndex* tip = b.Tip();
            CBlockUndo undo;
            REQUIRE(UndoReadFromDisk(undo, tip->GetUndoPos(), tip->pprev->GetBlockHash()));
            r.undo = SerializeToBytes(undo, SER_DISK, PROTOCOL_VERSION);
        }
        const std::string cmd = std::string("rm -rf '") + tmpl + "'";
        if (system(cmd.c_str()) != 0) {}
    }
    // serial (par 0) and parallel (par 1) runs; within each, Verdicts ran both passes too
    CHECK_EQ(res[0].fast, (int64_t)0);
    CHECK_EQ(res[1].fast, (int64_t)1);
    for (const Result& r : res) {
        CHECK_EQ(r.verdict.first, std::string("valid"));
        CHECK_EQ(r.verdict.second, std::string("valid"));
        CHECK_EQ(r.badVerdict.first, std::string("bad-txns-inputs-missingorspent"));
        CHECK_EQ(r.badVerdict.second, r.badVerdict.first);
    }
    CHECK(Same(res[0].coins, res[1].coins));
    // the coinbase's output replaced the old coin (height and value of the new block)
    CHECK(res[1].coins.at(cbOut.ToString()).find("/7/") == std::string::npos);
    CHECK(!res[1].coins.at(cbOut.ToString()).empty());
    CHECK(res[0].undo == res[1].undo);
    CHECK_EQ(res[0].undo.size() > 0, true);
}

// The connect lookahead: while block N's signature batch is out (here the GPU path with every
// batch failing over to the CPU, -gpufaultinjection), block N+1's read-only pass runs on the
// script threads against the tip N left. Four 1100-transaction blocks connected last-to-first in
// one ActivateBestChain: the later ones adopt their lookahead, and the chain and coins are the
// same as the node that connected them one by one without it.
TEST_CASE(connectblock_tests, lookahead_adopted_and_same_coins) {
    test::TestChain100Setup setup;
    Chainstate& a = *setup.node->chainstate;
    const CKey& key = setup.coinbaseKey;
    const CScript spk = P2PK(key);
    std::vector<CMutableTransaction> all;
    const size_t W = 1100;
    const Amount each = (setup.coinbaseTxns[0].vout[0].nValue - 100000) / (Amount)W;
    all.push_back(Make({{setup.coinbaseTxns[0], 0}}, std::vector<CTxOut>(W, CTxOut(each, spk)), key));
    setup.CreateAndProcessBlock({all[0]}, spk);
    std::vector<Prev> outs;
    {
        const CTransaction fan(all[0]);
        for (uint32_t i = 0; i < W; i++) outs.push_back({fan, i});
    }
    for (int b = 0; b < 4; b++) {
        std::vector<CMutableTransaction> txs;
        std::vector<Prev> next;
        for (size_t i = 0; i < W; i++) {
            const Amount v = outs[i].tx.vout[outs[i].n].nValue;
            txs.push_back(Make({outs[i]}, {CTxOut(v - 500, spk)}, key));
            next.push_back({CTransaction(txs.back()), 0});
        }
        setup.CreateAndProcessBlock(txs, spk);
        all.insert(all.end(), txs.begin(), txs.end());
        outs.swap(next);
    }
    std::vector<std::shared_ptr<const CBlock>> chain;
    for (const CBlockIndex* p = a.TipNow(); p && p->pprev; p = p->pprev) {
        auto blk = std::make_shared<CBlock>();
        REQUIRE(ReadBlockFromDisk(*blk, p, Params(), true));
        chain.insert(chain.begin(), blk);
    }
    const size_t thr = GetGpuSigThreshold();
    SetGpuSigThreshold(1);
    SetGpuFaultInjection(true);
    ResetGpuSigFailures();
    struct Undo {
        size_t thr;
        ~Undo() {
            SetGpuFaultInjection(false);
            ResetGpuSigFailures();
            SetGpuSigThreshold(thr);
        }
    } undo{thr};
    ChainstateOptions o;
    o.memoryOnly = true;
    char tmpl[] = "/tmp/bcp_test_lookahead_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    o.datadir = tmpl;
    o.useGpu = true; // batches go the GPU way (and fail over to the CPU)
    Chainstate b(Params(), o);
    std::string err;
    REQUIRE(b.InitBlockIndex(err));
    auto feed = [&](const std::shared_ptr<const CBlock>& blk) {
        bool fNew = false;
        CValidationState st;
        return b.ProcessNewBlock(blk, true, &fNew, &st);
    };
    const size_t n = chain.size();
    for (size_t i = 0; i + 4 < n; i++) REQUIRE(feed(chain[i]));
    std::vector<CBlockHeader> hdrs;
    for (size_t i = n - 4; i < n; i++) hdrs.push_back(chain[i]->GetBlockHeader());
    CValidationState hs;
    REQUIRE(b.ProcessNewBlockHeaders(hdrs, hs));
    const int64_t used0 = b.ConnectPhaseMicros(Chainstate::PH_LA_USED);
    for (size_t i = n; i-- > n - 4;) REQUIRE(feed(chain[i])); // last to first
    CHECK(b.TipNow()->GetBlockHash() == a.TipNow()->GetBlockHash());
    // blocks 2 and 3 adopt the lookahead of the block before (after three failed GPU batches the
    // GPU path is off, so block 4 is not looked ahead)
    CHECK(b.ConnectPhaseMicros(Chainstate::PH_LA_USED) - used0 >= 2);
    std::map<std::string, std::string> sa, sb;
    {
        std::lock_guard<CCriticalSection> l(a.cs());
        sa = Snapshot(a, all, {});
    }
    {
        std::lock_guard<CCriticalSection> l(b.cs());
        sb = Snapshot(b, all, {});
    }
    CHECK(Same(sa, sb));
    {
        // their undo records (serialised and checksummed beside the batch) read back
        std::lock_guard<CCriticalSection> l(b.cs());
        int k = 0;
        for (const CBlockIndex* p = b.Tip(); k < 4; p = p->pprev, k++) {
            CBlockUndo u;
            CHECK(UndoReadFromDisk(u, p->GetUndoPos(), p->pprev->GetBlockHash()));
            CHECK_EQ(u.vtxundo.size(), W);
        }
    }
    const std::string cmd = std::string("rm -rf '") + tmpl + "'";
    if (system(cmd.c_str()) != 0) {}
}

// Blocks accepted out of order connect from the recent-block cache (no disk read, no second
// CheckBlock), and the chain is the same with the cache off (-blockcachemb=0 reads them back).
TEST_CASE(connectblock_tests, recent_block_cache_out_of_order) {
    test::TestChain100Setup setup;
    Chainstate& a = *setup.node->chainstate;
    const CScript spk = P2PK(setup.coinbaseKey);
    for (int i = 0; i < 3; i++) setup.CreateAndProcessBlock({}, spk);
    std::vector<std::shared_ptr<const CBlock>> chain; // a's blocks above genesis, in height order
    for (const CBlockIndex* p = a.TipNow(); p && p->pprev; p = p->pprev) {
        auto b = std::make_shared<CBlock>();
        REQUIRE(ReadBlockFromDisk(*b, p, Params(), true));
        chain.insert(chain.begin(), b);
    }
    REQUIRE(chain.size() >= 4);
    for (size_t cacheBytes : {(size_t)64 << 20, (size_t)0}) {
        ChainstateOptions o;
        o.memoryOnly = true;
        char tmpl[] = "/tmp/bcp_test_recent_XXXXXX";
        REQUIRE(mkdtemp(tmpl) != nullptr);
        o.datadir = tmpl;
        o.useGpu = false;
        o.recentBlockBytes = cacheBytes;
        Chainstate b(Params(), o);
        std::string err;
        REQUIRE(b.InitBlockIndex(err));
        auto feed = [&](const std::shared_ptr<const CBlock>& blk) {
            bool fNew = false;
            CValidationState st;
            return b.ProcessNewBlock(blk, true, &fNew, &st);
        };
        const size_t n = chain.size();
        for (size_t i = 0; i + 3 < n; i++) REQUIRE(feed(chain[i]));
        std::vector<CBlockHeader> hdrs;
        for (size_t i = n - 3; i < n; i++) hdrs.push_back(chain[i]->GetBlockHeader());
        CValidationState hs;
        REQUIRE(b.ProcessNewBlockHeaders(hdrs, hs));
        const uint64_t h0 = b.RecentBlockHits(), m0 = b.RecentBlockMisses();
        for (size_t i = n; i-- > n - 3;) REQUIRE(feed(chain[i])); // last to first
        CHECK(b.TipNow()->GetBlockHash() == a.TipNow()->GetBlockHash());
        // the step connects all three after the last one arrives; ConnectTip gets none of them
        // as its argument (it is not the most-work block)
        CHECK_EQ(b.RecentBlockHits() - h0, cacheBytes ? (uint64_t)3 : (uint64_t)0);
        CHECK_EQ(b.RecentBlockMisses() - m0, cacheBytes ? (uint64_t)0 : (uint64_t)3);
        const std::string cmd = std::string("rm -rf '") + tmpl + "'";
        if (system(cmd.c_str()) != 0) {}
    }
}

// The parallel undo serialiser writes the same bytes as the plain serialiser (the on-disk
// record's checksum and every later DisconnectBlock depend on it).
TEST_CASE(connectblock_tests, undo_serialisation_parallel_matches) {
    std::mt19937_64 rng(7);
    CBlockUndo undo;
    undo.vtxundo.resize(5000);
    for (CTxUndo& tu : undo.vtxundo) {
        tu.vprevout.resize(1 + rng() % 3);
        for (Coin& c : tu.vprevout) {
            c.nHeight = (uint32_t)(rng() % 700000);
            c.fCoinBase = rng() % 7 == 0;
            c.out.nValue = (Amount)(rng() % 2100000000000000ULL);
            std::vector<unsigned char> h(20);
            for (auto& b : h) b = (unsigned char)rng();
            if (rng() % 4) c.out.scriptPubKey = CScript() << OP_DUP << OP_HASH160 << h << OP_EQUALVERIFY << OP_CHECKSIG;
            else c.out.scriptPubKey = CScript() << OP_RETURN << std::vector<unsigned char>(rng() % 80, 0xab);
        }
    }
    WorkerPool pool(4);
    const std::vector<unsigned char> plain = SerializeToBytes(undo, SER_DISK, PROTOCOL_VERSION);
    CHECK(SerializeBlockUndo(undo, &pool) == plain);
    CHECK(SerializeBlockUndo(undo, nullptr) == plain);
    CBlockUndo small;
    small.vtxundo.assign(undo.vtxundo.begin(), undo.vtxundo.begin() + 10);
    CHECK(SerializeBlockUndo(small, &pool) == SerializeToBytes(small, SER_DISK, PROTOCOL_VERSION));
}
