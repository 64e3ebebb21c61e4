// Relay data-structure suites: BIP37 bloom filters, partial merkle trees, BIP152 compact blocks.
// Parity:
//   bloom_tests           reference src/test/bloom_tests.cpp (filter serialization golden vectors
//                         incl. tweak and a key/pubkey-hash filter, IsRelevantAndUpdate outpoint
//                         tracking, CMerkleBlock matching, CRollingBloomFilter generations)
//   pmt_tests             reference src/test/pmt_tests.cpp (build/serialize/extract partial merkle
//                         trees for random match sets over many block sizes; CVE-2012-2459 style
//                         duplicated-txid malleability is detected)
//   blockencodings_tests  reference src/test/blockencodings_tests.cpp (compact block round trips
//                         from a mempool, prefilled non-coinbase transactions, empty blocks,
//                         BlockTransactionsRequest differential encoding)
#include "test/unittest.h"

#include "consensus/merkle.h"
#include "consensus/merkleblock.h"
#include "net/blockencodings.h"
#include "node/txmempool.h"
#include "primitives/serialize.h"
#include "script/standard.h"
#include "util/strencodings.h"

#include <random>
#include <set>

using namespace bcp;
using namespace bcp::test;

static std::string SerHex(const CBloomFilter& f) {
    std::vector<unsigned char> v;
    VectorWriter w(v);
    w << f;
    return HexStr(v.begin(), v.end());
}

// ------------------------------------------------------------------ bloom_tests

TEST_CASE(bloom_tests, create_insert_serialize) {
    BasicTestingSetup setup;
    CBloomFilter f(3, 0.01, 0, 1 /*BLOOM_UPDATE_ALL*/);
    f.insert(ParseHex("99108ad8ed9bb6274d3980bab5a85c048f0950c8"));
    CHECK(f.contains(ParseHex("99108ad8ed9bb6274d3980bab5a85c048f0950c8")));
    CHECK(!f.contains(ParseHex("19108ad8ed9bb6274d3980bab5a85c048f0950c8"))); // one bit off
    f.insert(ParseHex("b5a2c786d9ef4658287ced5914b37a1b4aa32eee"));
    CHECK(f.contains(ParseHex("b5a2c786d9ef4658287ced5914b37a1b4aa32eee")));
    f.insert(ParseHex("b9300670b4c5366e95b2699e8b18bc75e5f729c5"));
    CHECK(f.contains(ParseHex("b9300670b4c5366e95b2699e8b18bc75e5f729c5")));
    CHECK_EQ(SerHex(f), std::string("03614e9b050000000000000001"));
    f.clear();
    CHECK(!f.contains(ParseHex("99108ad8ed9bb6274d3980bab5a85c048f0950c8")));
}

TEST_CASE(bloom_tests, create_insert_serialize_with_tweak) {
    BasicTestingSetup setup;
    CBloomFilter f(3, 0.01, 2147483649UL, 1);
    for (const char* h : {"99108ad8ed9bb6274d3980bab5a85c048f0950c8", "b5a2c786d9ef4658287ced5914b37a1b4aa32eee",
                          "b9300670b4c5366e95b2699e8b18bc75e5f729c5"}) {
        f.insert(ParseHex(h));
        CHECK(f.contains(ParseHex(h)));
    }
    CHECK(!f.contains(ParseHex("19108ad8ed9bb6274d3980bab5a85c048f0950c8")));
    CHECK_EQ(SerHex(f), std::string("03ce4299050000000100008001"));
}

TEST_CASE(bloom_tests, create_insert_key) {
    BasicTestingSetup setup("main");
    CKey key = DecodeSecret("5Kg1gnAjaLfKiwhhPpGS3QfRg2m6awQvaj98JCZBZQ5SuS2F15C", Params());
    REQUIRE(key.IsValid());
    CPubKey pub = key.GetPubKey();
    CBloomFilter f(2, 0.001, 0, 1);
    f.insert(pub.Raw());
    const uint160 id = pub.GetID();
    f.insert(std::vector<unsigned char>(id.begin(), id.end()));
    CHECK_EQ(SerHex(f), std::string("038fc16b080000000000000001"));
}

static CMutableTransaction SpendTx(const uint256& prev, uint32_t n, const CScript& spk, Amount v = 1000) {
    CMutableTransaction t;
    t.nVersion = 1;
    t.vin.resize(1);
    t.vin[0].prevout = COutPoint(prev, n);
    t.vin[0].scriptSig = CScript() << std::vector<unsigned char>(71, 0x30) << std::vector<unsigned char>(33, 0x02);
    t.vout.push_back(CTxOut(v, spk));
    return t;
}

TEST_CASE(bloom_tests, match_and_update) {
    BasicTestingSetup setup;
    CKey k;
    k.MakeNewKey(true);
    const CScript p2pk = CScript() << k.GetPubKey().Raw() << OP_CHECKSIG;
    const CScript p2pkh = GetScriptForDestination(k.GetPubKey().GetID());
    const CTransaction tx0(SpendTx(GetRandHash(), 0, p2pk));
    const CTransaction spend0(SpendTx(tx0.GetHash(), 0, CScript() << OP_TRUE));
    const CTransaction unrelated(SpendTx(GetRandHash(), 3, CScript() << OP_TRUE));
    {
        CBloomFilter f(10, 0.000001, 0, 1 /*UPDATE_ALL*/);
        f.insert(tx0.GetHash());
        CHECK(f.IsRelevantAndUpdate(tx0)); // by txid
        CHECK(!f.IsRelevantAndUpdate(unrelated));
    }
    {
        // a data push of an output matches and, with UPDATE_ALL, the outpoint is added so the
        // spending transaction matches too
        CBloomFilter f(10, 0.000001, 0, 1);
        f.insert(k.GetPubKey().Raw());
        CHECK(f.IsRelevantAndUpdate(tx0));
        CHECK(f.contains(COutPoint(tx0.GetHash(), 0)));
        CHECK(f.IsRelevantAndUpdate(spend0));
    }
    {
        // UPDATE_NONE: the output matches but its outpoint is not added
        CBloomFilter f(10, 0.000001, 0, 0);
        f.insert(k.GetPubKey().Raw());
        CHECK(f.IsRelevantAndUpdate(tx0));
        CHECK(!f.IsRelevantAndUpdate(spend0));
    }
    {
        // UPDATE_P2PUBKEY_ONLY (2): pay-to-pubkey outputs are added, pay-to-pubkey-hash ones are not
        const CTransaction txh(SpendTx(GetRandHash(), 0, p2pkh));
        const CTransaction spendh(SpendTx(txh.GetHash(), 0, CScript() << OP_TRUE));
        CBloomFilter f(10, 0.000001, 0, 2);
        const uint160 id = k.GetPubKey().GetID();
        f.insert(k.GetPubKey().Raw());
        f.insert(std::vector<unsigned char>(id.begin(), id.end()));
        CHECK(f.IsRelevantAndUpdate(tx0));
        CHECK(f.IsRelevantAndUpdate(spend0));
        CHECK(f.IsRelevantAndUpdate(txh));
        CHECK(!f.IsRelevantAndUpdate(spendh));
    }
    {
        // an input's scriptSig data or prevout matches
        CBloomFilter f(10, 0.000001, 0, 1);
        f.insert(COutPoint(unrelated.vin[0].prevout));
        CHECK(f.IsRelevantAndUpdate(unrelated));
        CBloomFilter g(10, 0.000001, 0, 1);
        g.insert(std::vector<unsigned char>(33, 0x02));
        CHECK(g.IsRelevantAndUpdate(unrelated));
    }
}

static CBlock MakeBlock(int ntx, std::mt19937& rng) {
    CBlock b;
    b.nVersion = 4;
    b.nTime = 1500000000;
    b.nBits = 0x207fffff;
    for (int i = 0; i < ntx; i++) {
        CMutableTransaction t;
        t.nVersion = 1;
        t.vin.resize(1);
        uint256 h;
        for (int j = 0; j < 32; j++) h.begin()[j] = (unsigned char)rng();
        t.vin[0].prevout = COutPoint(h, (uint32_t)i);
        t.vout.push_back(CTxOut(i + 1, CScript() << OP_TRUE));
        b.vtx.push_back(MakeTransactionRef(t));
    }
    b.hashMerkleRoot = BlockMerkleRoot(b);
    return b;
}

TEST_CASE(bloom_tests, merkle_block_matches) {
    BasicTestingSetup setup;
    std::mt19937 rng(7);
    CBlock block = MakeBlock(9, rng);
    std::set<uint256> want = {block.vtx[2]->GetHash(), block.vtx[7]->GetHash()};
    CBloomFilter f(10, 0.000001, 0, 0);
    for (const uint256& h : want) f.insert(h);
    CMerkleBlock mb(block, f);
    CHECK(mb.header.GetHash() == block.GetHash());
    REQUIRE(mb.vMatchedTxn.size() == 2);
    CHECK(mb.vMatchedTxn[0].first == 2 && mb.vMatchedTxn[0].second == block.vtx[2]->GetHash());
    CHECK(mb.vMatchedTxn[1].first == 7 && mb.vMatchedTxn[1].second == block.vtx[7]->GetHash());
    std::vector<uint256> matched;
    std::vector<unsigned> idx;
    CHECK(mb.txn.ExtractMatches(matched, idx) == block.hashMerkleRoot);
    CHECK(matched.size() == 2 && idx[0] == 2 && idx[1] == 7);
    // serialization round trip
    std::vector<unsigned char> v;
    VectorWriter w(v);
    w << mb;
    CMerkleBlock mb2;
    SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
    r >> mb2;
    std::vector<uint256> m2;
    std::vector<unsigned> i2;
    CHECK(mb2.txn.ExtractMatches(m2, i2) == block.hashMerkleRoot && m2 == matched && i2 == idx);
    // txid-set constructor (gettxoutproof)
    CMerkleBlock mb3(block, want);
    std::vector<uint256> m3;
    std::vector<unsigned> i3;
    CHECK(mb3.txn.ExtractMatches(m3, i3) == block.hashMerkleRoot && m3 == matched);
}

TEST_CASE(bloom_tests, rolling_bloom) {
    BasicTestingSetup setup;
    std::mt19937 rng(99);
    auto rnd = [&]() {
        std::vector<unsigned char> d(32);
        for (auto& c : d) c = (unsigned char)rng();
        return d;
    };
    CRollingBloomFilter rb1(100, 0.01);
    const int N = 399;
    std::vector<std::vector<unsigned char>> data(N);
    for (int i = 0; i < N; i++) {
        data[i] = rnd();
        rb1.insert(data[i]);
    }
    for (int i = 299; i < N; i++) CHECK(rb1.contains(data[i])); // last 100 remembered
    unsigned hits = 0;
    for (int i = 0; i < 10000; i++) hits += rb1.contains(rnd());
    CHECK(hits > 25 && hits < 175); // ~1% false positives
    CHECK(rb1.contains(data[N - 1]));
    rb1.reset();
    CHECK(!rb1.contains(data[N - 1]));
    for (int i = 0; i < N; i++) {
        if (i >= 100) CHECK(rb1.contains(data[i - 100]));
        rb1.insert(data[i]);
        CHECK(rb1.contains(data[i]));
    }
    for (int i = 0; i < 999; i++) {
        auto d = rnd();
        rb1.insert(d);
        CHECK(rb1.contains(d));
    }
    hits = 0;
    for (int i = 0; i < N; i++) hits += rb1.contains(data[i]);
    CHECK(hits < 100);
    CRollingBloomFilter rb2(1000, 0.001);
    for (int i = 0; i < N; i++) rb2.insert(data[i]);
    for (int i = 0; i < N; i++) CHECK(rb2.contains(data[i]));
}

// ------------------------------------------------------------------ pmt_tests

// Partial tree whose serialized form is read back from bytes (so fBad starts cleared).
static CPartialMerkleTree RoundTrip(const CPartialMerkleTree& t) {
    std::vector<unsigned char> v;
    VectorWriter w(v);
    w << t;
    CPartialMerkleTree t2;
    SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
    r >> t2;
    return t2;
}

TEST_CASE(pmt_tests, build_extract_random) {
    BasicTestingSetup setup;
    std::mt19937 rng(31337);
    const unsigned sizes[] = {1, 4, 7, 17, 56, 100, 127, 256, 312, 513, 1000, 4095};
    for (unsigned ntx : sizes) {
        CBlock block = MakeBlock((int)ntx, rng);
        std::vector<uint256> txids;
        for (const auto& t : block.vtx) txids.push_back(t->GetHash());
        const uint256 root = BlockMerkleRoot(block);
        for (int att = 1; att < 15; att++) {
            // match roughly 1 in 2^(att/2) transactions
            std::vector<bool> match(ntx, false);
            std::vector<uint256> wantTx;
            std::vector<unsigned> wantIdx;
            for (unsigned j = 0; j < ntx; j++) {
                const bool inc = (rng() & ((1u << (att / 2)) - 1)) == 0;
                match[j] = inc;
                if (inc) {
                    wantTx.push_back(txids[j]);
                    wantIdx.push_back(j);
                }
            }
            CPartialMerkleTree pmt1(txids, match);
            // the encoding stays within the reference bound: ~ n*log2(ntx/n) hashes
            CPartialMerkleTree pmt2 = RoundTrip(pmt1);
            std::vector<uint256> got;
            std::vector<unsigned> idx;
            const uint256 r2 = pmt2.ExtractMatches(got, idx);
            CHECK(r2 == root);
            CHECK(got == wantTx);
            CHECK(idx == wantIdx);
            CHECK_EQ(pmt2.GetNumTransactions(), ntx);
        }
    }
}

TEST_CASE(pmt_tests, malleability) {
    BasicTestingSetup setup;
    // txids 9 and 10 equal 8 and 9's partners would collide the tree: duplicated last hashes
    std::vector<uint256> v;
    for (int i = 1; i <= 12; i++) v.push_back(ArithToUint256(arith_uint256(i)));
    v[9] = v[8];
    v[11] = v[10];
    std::vector<bool> match = {false, false, false, false, false, false, false, false, false, true, true, false};
    CPartialMerkleTree tree(v, match);
    std::vector<uint256> got;
    std::vector<unsigned> idx;
    CHECK(tree.ExtractMatches(got, idx).IsNull()); // mutated tree rejected
}

// ------------------------------------------------------------------ blockencodings_tests

static CMutableTransaction FeeTx(const uint256& prev, Amount out) {
    CMutableTransaction t;
    t.nVersion = 1;
    t.vin.resize(1);
    t.vin[0].prevout = COutPoint(prev, 0);
    t.vin[0].scriptSig = CScript() << OP_11;
    t.vout.push_back(CTxOut(out, CScript() << OP_11 << OP_EQUAL));
    return t;
}

// coinbase + tx1 + tx2 (+ tx3), with a valid merkle root (no PoW needed here)
static CBlock BuildBlock3() {
    CBlock b;
    CMutableTransaction cb;
    cb.vin.resize(1);
    cb.vin[0].prevout.SetNull();
    cb.vin[0].scriptSig = CScript() << 42 << OP_TRUE;
    cb.vout.push_back(CTxOut(50 * COIN, CScript() << OP_TRUE));
    b.vtx.push_back(MakeTransactionRef(cb));
    uint256 prev = GetRandHash();
    for (int i = 0; i < 3; i++) {
        CMutableTransaction t = FeeTx(prev, 1000 * (i + 1));
        b.vtx.push_back(MakeTransactionRef(t));
        prev = b.vtx.back()->GetHash();
    }
    b.nVersion = 4;
    b.nBits = 0x207fffff;
    b.hashMerkleRoot = BlockMerkleRoot(b);
    return b;
}

static void AddToPool(CTxMemPool& pool, const CTransactionRef& tx) {
    LockPoints lp;
    CTxMemPoolEntry e(tx, 1000, 0, 0.0, 1, 0, false, 1, lp);
    std::lock_guard<CCriticalSection> l(pool.cs);
    pool.addUnchecked(tx->GetHash(), e);
}

TEST_CASE(blockencodings_tests, SimpleRoundTrip) {
    TestingSetup setup;
    CTxMemPool pool;
    CBlock block = BuildBlock3();
    AddToPool(pool, block.vtx[2]);
    CBlockHeaderAndShortTxIDs cmpct(block, 0x1234);
    // serialize / deserialize
    std::vector<unsigned char> v;
    VectorWriter w(v);
    w << cmpct;
    CBlockHeaderAndShortTxIDs c2;
    SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
    r >> c2;
    PartiallyDownloadedBlock part(&pool);
    REQUIRE(part.InitData(c2, {}) == READ_STATUS_OK);
    CHECK(part.IsTxAvailable(0));  // coinbase prefilled
    CHECK(!part.IsTxAvailable(1));
    CHECK(part.IsTxAvailable(2));  // from the mempool
    CHECK(!part.IsTxAvailable(3));
    CBlock out;
    // wrong transactions for the missing slots: the merkle re-check refuses the block (corruption
    // possible -> READ_STATUS_FAILED, reference blockencodings.cpp FillBlock)
    CHECK(part.FillBlock(out, {block.vtx[3], block.vtx[1]}) == READ_STATUS_FAILED);
    PartiallyDownloadedBlock part2(&pool);
    REQUIRE(part2.InitData(c2, {}) == READ_STATUS_OK);
    CBlock out2;
    CHECK(part2.FillBlock(out2, {block.vtx[1], block.vtx[3]}) == READ_STATUS_OK);
    CHECK(out2.GetHash() == block.GetHash());
    CHECK(BlockMerkleRoot(out2) == block.hashMerkleRoot);
    // too few transactions supplied
    PartiallyDownloadedBlock part3(&pool);
    REQUIRE(part3.InitData(c2, {}) == READ_STATUS_OK);
    CBlock out3;
    CHECK(part3.FillBlock(out3, {block.vtx[1]}) == READ_STATUS_INVALID);
}

TEST_CASE(blockencodings_tests, ExtraPoolAndPrefilled) {
    TestingSetup setup;
    CTxMemPool pool;
    CBlock block = BuildBlock3();
    // a compact block with a non-coinbase prefilled transaction; tx2 comes from the extra pool
    CBlockHeaderAndShortTxIDs cmpct(block, 99);
    cmpct.prefilledtxn.push_back({3, block.vtx[3]});
    cmpct.shorttxids.pop_back(); // shortids of vtx 1, 2 only
    std::vector<std::pair<uint256, CTransactionRef>> extra = {{block.vtx[2]->GetHash(), block.vtx[2]}};
    PartiallyDownloadedBlock part(&pool);
    REQUIRE(part.InitData(cmpct, extra) == READ_STATUS_OK);
    CHECK(part.IsTxAvailable(0) && !part.IsTxAvailable(1) && part.IsTxAvailable(2) && part.IsTxAvailable(3));
    CBlock out;
    CHECK(part.FillBlock(out, {block.vtx[1]}) == READ_STATUS_OK);
    CHECK(out.GetHash() == block.GetHash() && out.vtx.size() == 4);
}

TEST_CASE(blockencodings_tests, EmptyBlockRoundTrip) {
    TestingSetup setup;
    CTxMemPool pool;
    CBlock block = BuildBlock3();
    block.vtx.resize(1);
    block.hashMerkleRoot = BlockMerkleRoot(block);
    CBlockHeaderAndShortTxIDs cmpct(block, 5);
    CHECK(cmpct.shorttxids.empty() && cmpct.prefilledtxn.size() == 1);
    PartiallyDownloadedBlock part(&pool);
    REQUIRE(part.InitData(cmpct, {}) == READ_STATUS_OK);
    CBlock out;
    CHECK(part.FillBlock(out, {}) == READ_STATUS_OK);
    CHECK(out.GetHash() == block.GetHash());
}

TEST_CASE(blockencodings_tests, TransactionsRequestSerialization) {
    BasicTestingSetup setup;
    BlockTransactionsRequest req;
    req.blockhash = GetRandHash();
    req.indexes = {0, 1, 3, 4};
    std::vector<unsigned char> v;
    VectorWriter w(v);
    w << req;
    // differential indexes on the wire: 0, 0, 1, 0
    CHECK_EQ(HexStr(v.begin() + 32, v.end()), std::string("0400000100"));
    BlockTransactionsRequest req2;
    SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
    r >> req2;
    CHECK(req2.blockhash == req.blockhash);
    CHECK(req2.indexes == req.indexes);
}
