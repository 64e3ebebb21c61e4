// miner_tests, policyestimator_tests and txvalidationcache_tests.
// Parity: reference src/test/miner_tests.cpp (CreateNewBlock: package selection - a high-fee
// child pulls its low-fee parent in, parents before children -, fee accounting in the coinbase,
// non-final transactions left out, size and sigop limits respected, the template passes
// TestBlockValidity), src/test/policyestimator_tests.cpp (BlockPolicyEstimates: fee levels that
// confirm after known delays give monotone estimates near those levels; no data -> no estimate;
// decay; persistence) and src/test/txvalidationcache_tests.cpp (mempool -> block, a block that
// double-spends a mempool transaction evicts it, and script-validation results are never reused
// across different flag sets: a high-S signature refused by the mempool is still valid in a
// pre-fork block).
#include "test/unittest.h"

#include "consensus/tx_verify.h"
#include "node/miner.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "script/sign.h"
#include "util/strencodings.h"

#include <cstdio>
#include <deque>

using namespace bcp;

namespace {

CScript P2PK(const CKey& k) { return CScript() << k.GetPubKey().Raw() << OP_CHECKSIG; }

// spend output `n` of `prev` (P2PK to `key`) into `nOut` equal outputs, paying `fee`
CMutableTransaction Spend(const CTransaction& prev, uint32_t n, const CKey& key, Amount fee, int nOut = 1,
                          uint32_t nLockTime = 0, uint32_t nSequence = CTxIn::SEQUENCE_FINAL) {
    CMutableTransaction m;
    m.nLockTime = nLockTime;
    m.vin.push_back(CTxIn(COutPoint(prev.GetHash(), n), CScript(), nSequence));
    const Amount each = (prev.vout[n].nValue - fee) / nOut;
    for (int i = 0; i < nOut; i++) m.vout.push_back(CTxOut(each, P2PK(key)));
    CBasicKeyStore ks;
    ks.AddKey(key);
    if (!SignSignature(ks, prev.vout[n].scriptPubKey, m, 0, prev.vout[n].nValue, SIGHASH_ALL | SIGHASH_FORKID))
        throw std::runtime_error("test: signing failed");
    return m;
}

bool Accept(Chainstate& cs, const CMutableTransaction& m, std::string* reason = nullptr) {
    CValidationState st;
    bool missing = false;
    const bool ok = cs.AcceptToMemoryPool(st, MakeTransactionRef(m), false, &missing, true);
    if (reason) *reason = st.GetRejectReason();
    return ok;
}

std::unique_ptr<CBlockTemplate> Template(NodeContext& node, const CScript& spk,
                                         const BlockAssembler::Options& o = BlockAssembler::Options()) {
    BlockAssembler ba(*node.chainstate, node.mempool.get(), o);
    return ba.CreateNewBlock(spk);
}

// s -> n - s in a DER signature (the other, "high" S of the same signature)
std::vector<unsigned char> HighS(const std::vector<unsigned char>& der) {
    static const unsigned char N[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                        0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                                        0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};
    const size_t rlen = der[3];
    std::vector<unsigned char> r(der.begin() + 4, der.begin() + 4 + rlen);
    const size_t slen = der[5 + rlen];
    std::vector<unsigned char> s(der.begin() + 6 + rlen, der.begin() + 6 + rlen + slen);
    while (!s.empty() && s[0] == 0) s.erase(s.begin());
    unsigned char s32[32] = {0}, h[32];
    memcpy(s32 + 32 - s.size(), s.data(), s.size());
    int borrow = 0;
    for (int i = 31; i >= 0; i--) {
        int d = (int)N[i] - s32[i] - borrow;
        borrow = d < 0;
        h[i] = (unsigned char)(d + (borrow ? 256 : 0));
    }
    std::vector<unsigned char> hs(h, h + 32);
    while (hs.size() > 1 && hs[0] == 0 && !(hs[1] & 0x80)) hs.erase(hs.begin());
    if (hs[0] & 0x80) hs.insert(hs.begin(), 0);
    std::vector<unsigned char> out{0x30, 0, 0x02, (unsigned char)r.size()};
    out.insert(out.end(), r.begin(), r.end());
    out.push_back(0x02);
    out.push_back((unsigned char)hs.size());
    out.insert(out.end(), hs.begin(), hs.end());
    out[1] = (unsigned char)(out.size() - 2);
    return out;
}

} // namespace

// ------------------------------------------------------------------ miner_tests
// coinbases 0..n-1 of the fixture spendable (COINBASE_MATURITY more blocks on top of each)
static void Mature(test::TestChain100Setup& setup, int n) {
    for (int i = 1; i < n; i++) setup.CreateAndProcessBlock({}, P2PK(setup.coinbaseKey));
}

TEST_CASE(miner_tests, package_selection_and_fees) {
    test::TestChain100Setup setup;
    Mature(setup, 2);
    NodeContext& node = *setup.node;
    Chainstate& cs = *node.chainstate;
    const CKey& key = setup.coinbaseKey;
    // parent pays almost nothing, its child a lot: mined together, parent first; an independent
    // medium-fee transaction sorts between the package and nothing else
    const CMutableTransaction parent = Spend(setup.coinbaseTxns[0], 0, key, 1000);
    const CMutableTransaction child = Spend(CTransaction(parent), 0, key, 4000000);
    const CMutableTransaction other = Spend(setup.coinbaseTxns[1], 0, key, 200000);
    REQUIRE(Accept(cs, parent));
    REQUIRE(Accept(cs, child));
    REQUIRE(Accept(cs, other));
    BlockAssembler::Options byFee; // no priority area: pure (package) feerate order
    byFee.nBlockPriorityPercentage = 0;
    std::unique_ptr<CBlockTemplate> t = Template(node, P2PK(key), byFee);
    REQUIRE(t->block.vtx.size() == 4);
    std::map<uint256, size_t> pos;
    for (size_t i = 0; i < t->block.vtx.size(); i++) pos[t->block.vtx[i]->GetHash()] = i;
    const uint256 hp = CTransaction(parent).GetHash(), hc = CTransaction(child).GetHash(), ho = CTransaction(other).GetHash();
    CHECK(pos.count(hp) && pos.count(hc) && pos.count(ho));
    CHECK(pos[hp] < pos[hc]);
    CHECK(pos[hc] < pos[ho]); // package feerate (parent+child) beats the medium one
    // coinbase = subsidy + all fees; per-tx fees recorded
    Amount fees = 0;
    for (size_t i = 1; i < t->vTxFees.size(); i++) fees += t->vTxFees[i];
    CHECK_EQ(fees, (Amount)(1000 + 4000000 + 200000));
    CHECK_EQ(t->block.vtx[0]->GetValueOut(), GetBlockSubsidy(cs.HeightNow() + 1, cs.Params().GetConsensus()) + fees);
    CHECK_EQ(t->vTxSigOpsCount.size(), t->block.vtx.size());
    // the template is a valid block
    CBlock b = t->block;
    unsigned extra = 0;
    IncrementExtraNonce(&b, cs.TipNow(), extra, cs.MaxBlockSize());
    CValidationState st;
    CHECK(cs.TestBlockValidity(st, b, cs.TipNow(), false, true));
}

TEST_CASE(miner_tests, nonfinal_excluded_and_limits) {
    test::TestChain100Setup setup;
    Mature(setup, 40);
    NodeContext& node = *setup.node;
    Chainstate& cs = *node.chainstate;
    const CKey& key = setup.coinbaseKey;
    // a time-locked transaction the mempool holds (prioritised past policy) is not mined until final
    const int h = cs.HeightNow();
    const CMutableTransaction locked = Spend(setup.coinbaseTxns[2], 0, key, 50000, 1, (uint32_t)(h + 5), 0);
    std::string why;
    CHECK(!Accept(cs, locked, &why)); // the mempool refuses non-final transactions
    CHECK_EQ(why, std::string("bad-txns-nonfinal"));
    // many transactions: a small block size limit is respected
    for (int i = 3; i < 40; i++) REQUIRE(Accept(cs, Spend(setup.coinbaseTxns[i], 0, key, 10000 + i * 100, 20)));
    BlockAssembler::Options small;
    small.nMaxGeneratedBlockSize = 4000;
    std::unique_ptr<CBlockTemplate> t = Template(node, P2PK(key), small);
    CHECK(GetSerializeSize(t->block, PROTOCOL_VERSION) <= 4000);
    CHECK(t->block.vtx.size() > 1);
    CHECK(t->block.vtx.size() < 38);
    // a full-size template takes everything, sigops counted per transaction; with no priority
    // area (-blockprioritysize=0) it is ordered by feerate
    BlockAssembler::Options byFee;
    byFee.nBlockPriorityPercentage = 0;
    std::unique_ptr<CBlockTemplate> all = Template(node, P2PK(key), byFee);
    CHECK_EQ(all->block.vtx.size(), (size_t)38);
    int64_t sigops = 0;
    for (int64_t s : all->vTxSigOpsCount) sigops += s;
    CHECK(sigops <= (int64_t)GetMaxBlockSigOpsCount(GetSerializeSize(all->block, PROTOCOL_VERSION)));
    // highest feerates first among independent transactions
    for (size_t i = 2; i < all->block.vtx.size(); i++)
        CHECK(all->vTxFees[i - 1] * (Amount)GetSerializeSize(*all->block.vtx[i], PROTOCOL_VERSION) >=
              all->vTxFees[i] * (Amount)GetSerializeSize(*all->block.vtx[i - 1], PROTOCOL_VERSION));
}

// ------------------------------------------------------------------ policyestimator_tests
TEST_CASE(policyestimator_tests, fee_levels_with_known_delays) {
    // fee level k (k = 0..9, 1000*(k+1) sat/kB) always confirms after 10 - k blocks: the
    // estimate for target t is the cheapest level that confirms within t blocks
    CBlockPolicyEstimator est;
    CHECK_EQ(est.estimateFee(1).GetFeePerK(), 0); // no data: no estimate
    std::deque<std::pair<unsigned, uint256>> due[10];
    uint64_t nonce = 0;
    for (unsigned height = 1; height <= 400; height++) {
        std::vector<uint256> confirmed;
        for (int k = 0; k < 10; k++) {
            while (!due[k].empty() && due[k].front().first <= height) {
                confirmed.push_back(due[k].front().second);
                due[k].pop_front();
            }
        }
        est.processBlock(height, confirmed);
        for (int k = 0; k < 10; k++) {
            for (int i = 0; i < 5; i++) {
                uint256 h;
                const uint64_t v = ++nonce;
                memcpy(h.begin(), &v, 8);
                est.processTransaction(h, CFeeRate(1000 * (k + 1)), height, true);
                due[k].push_back({height + (unsigned)(10 - k), h});
            }
        }
    }
    Amount prev = INT64_MAX;
    for (int t = 1; t <= 10; t++) {
        const Amount e = est.estimateFee(t).GetFeePerK();
        const Amount level = 1000 * (10 - t + 1); // cheapest level confirming within t blocks
        CHECK(e >= level);
        CHECK(e <= level * 11 / 10 + 1); // one bucket (spacing 1.1) above at most
        CHECK(e <= prev);                // monotone in the target
        prev = e;
    }
    // beyond the slowest level nothing cheaper exists: same answer as t = 10
    CHECK_EQ(est.estimateFee(15).GetFeePerK(), est.estimateFee(10).GetFeePerK());
    // smart estimate: an unanswerable target falls back to the next one with an answer
    int found = 0;
    const CFeeRate s = est.estimateSmartFee(1, &found);
    CHECK_EQ(found, 1);
    CHECK_EQ(s.GetFeePerK(), est.estimateFee(1).GetFeePerK());
    // persistence round trip
    char tmpl[] = "/tmp/bcp_fees_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    const std::string path = std::string(tmpl) + "/fee_estimates.dat";
    REQUIRE(est.Write(path));
    CBlockPolicyEstimator back;
    REQUIRE(back.Read(path));
    for (int t = 1; t <= 12; t++) CHECK_EQ(back.estimateFee(t).GetFeePerK(), est.estimateFee(t).GetFeePerK());
    // a damaged file is refused (and leaves the estimator usable)
    FILE* f = fopen(path.c_str(), "r+b");
    REQUIRE(f != nullptr);
    fputc(0x7f, f);
    fclose(f);
    CBlockPolicyEstimator bad;
    CHECK(!bad.Read(path));
    CHECK_EQ(bad.estimateFee(1).GetFeePerK(), 0);
    const std::string cmd = std::string("rm -rf '") + tmpl + "'";
    if (system(cmd.c_str()) != 0) {}
    // with no new transactions the statistics decay until they no longer support an estimate
    unsigned height = 401;
    for (; height < 401 + 6000 && est.estimateFee(1).GetFeePerK() > 0; height++) est.processBlock(height, {});
    CHECK_EQ(est.estimateFee(1).GetFeePerK(), 0);
}

// ------------------------------------------------------------------ txvalidationcache_tests
TEST_CASE(txvalidationcache_tests, mempool_block_and_doublespend) {
    test::TestChain100Setup setup;
    Mature(setup, 2);
    NodeContext& node = *setup.node;
    Chainstate& cs = *node.chainstate;
    const CKey& key = setup.coinbaseKey;
    // accepted to the mempool, then mined: the block connects and the mempool empties
    const CMutableTransaction a = Spend(setup.coinbaseTxns[0], 0, key, 10000);
    REQUIRE(Accept(cs, a));
    setup.CreateAndProcessBlock({a}, P2PK(key));
    CHECK_EQ(node.mempool->size(), 0u);
    // a mempool spend of coin X, then a block with a different spend of X: the block wins and
    // evicts the mempool transaction (and nothing can re-add it)
    const CMutableTransaction x1 = Spend(setup.coinbaseTxns[1], 0, key, 10000);
    const CMutableTransaction x2 = Spend(setup.coinbaseTxns[1], 0, key, 20000);
    REQUIRE(Accept(cs, x1));
    setup.CreateAndProcessBlock({x2}, P2PK(key));
    CHECK(!node.mempool->exists(CTransaction(x1).GetHash()));
    CHECK(!Accept(cs, x1));
}

TEST_CASE(txvalidationcache_tests, results_not_shared_across_flags) {
    test::TestChain100Setup setup;
    NodeContext& node = *setup.node;
    Chainstate& cs = *node.chainstate;
    const CKey& key = setup.coinbaseKey;
    // the same spend with its signature's S flipped to the high half: LOW_S is a mempool (and
    // post-fork) rule, not a pre-fork block rule
    CMutableTransaction tx = Spend(setup.coinbaseTxns[0], 0, key, 10000);
    std::vector<unsigned char> sig(tx.vin[0].scriptSig.begin() + 1, tx.vin[0].scriptSig.end());
    const unsigned char ht = sig.back();
    sig.pop_back();
    std::vector<unsigned char> high = HighS(sig);
    high.push_back(ht);
    tx.vin[0].scriptSig = CScript() << high;
    std::string why;
    CHECK(!Accept(cs, tx, &why));
    CHECK(why.find("script-verify-flag-failed") != std::string::npos);
    // refusing it must not poison the block path: the pre-fork block with it connects
    const int before = cs.HeightNow();
    setup.CreateAndProcessBlock({tx}, P2PK(key));
    CHECK_EQ(cs.HeightNow(), before + 1);
    CHECK_EQ(node.mempool->size(), 0u);
}
