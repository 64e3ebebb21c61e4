// sigbatch_tests: deferred signature checking must decide exactly like eager script execution.
// Parity: the reference runs every CHECKSIG / CHECKMULTISIG eagerly (src/script/interpreter.cpp:
// 1008-1148); this node defers ECDSA into block-wide batches (DeferringSignatureChecker) and, for
// CHECKMULTISIG, speculatively records every (signature, key) pair the greedy match could try and
// replays the match over the batch results. A single divergent verdict would be a chain split, so
// randomized scripts are run both ways under the post-fork (NULLFAIL) flags and compared.
#include "test/unittest.h"

#include "keys/key.h"
#include "node/sigverify.h"
#include "script/interpreter.h"
#include "script/script.h"
#include "util/strencodings.h"

using namespace bcp;

namespace {

const uint32_t kFlags = STANDARD_SCRIPT_VERIFY_FLAGS; // NULLFAIL, STRICTENC, LOW_S, FORKID, NULLDUMMY
const Amount kAmount = 50000;

CMutableTransaction SpendOf(const CScript& spk) {
    CMutableTransaction credit;
    credit.vin.push_back(CTxIn(COutPoint(), CScript() << 0 << 0));
    credit.vout.push_back(CTxOut(kAmount, spk));
    CMutableTransaction spend;
    spend.vin.push_back(CTxIn(COutPoint(CTransaction(credit).GetHash(), 0)));
    spend.vout.push_back(CTxOut(kAmount - 1000, CScript() << OP_TRUE));
    return spend;
}

std::vector<unsigned char> SignFor(const CKey& key, const CScript& code, const CMutableTransaction& tx, uint32_t ht) {
    const uint256 h = SignatureHash(code, CTransaction(tx), 0, ht, kAmount, nullptr, kFlags);
    std::vector<unsigned char> sig;
    key.Sign(h, sig);
    sig.push_back((unsigned char)ht);
    return sig;
}

struct Outcome {
    bool eager, deferred;
    size_t groups, checks;
};

Outcome RunBoth(const CScript& scriptSig, const CScript& spk, const CMutableTransaction& mtx) {
    const CTransaction tx(mtx);
    Outcome o{};
    TransactionSignatureChecker eager(&tx, 0, kAmount);
    o.eager = VerifyScript(scriptSig, spk, kFlags, eager);
    std::vector<DeferredSigCheck> sink;
    std::vector<DeferredMultisig> groups;
    DeferringSignatureChecker lazy(&tx, 0, kAmount, nullptr, &sink, &groups);
    o.deferred = VerifyScript(scriptSig, spk, kFlags, lazy);
    if (o.deferred) o.deferred = BatchVerifySignatures(sink, groups, nullptr, false, false, false);
    o.groups = groups.size();
    o.checks = sink.size();
    return o;
}

} // namespace

TEST_CASE(sigbatch_tests, multisig_deferral_matches_eager) {
    test::BasicTestingSetup setup("main");
    FastRandomContext rng(true);
    std::vector<CKey> keys(20);
    for (size_t i = 0; i < keys.size(); i++) keys[i].MakeNewKey(i % 3 != 0);
    size_t deferredRuns = 0, valid = 0, invalid = 0;
    for (int trial = 0; trial < 1500; trial++) {
        const int n = 1 + (int)rng.randrange(trial % 10 == 0 ? 20 : 5);
        const int m = (int)rng.randrange(n + 1);
        // the key list: a random selection, sometimes with a key that fails STRICTENC
        std::vector<int> kidx(n);
        std::vector<std::vector<unsigned char>> pubs(n);
        for (int j = 0; j < n; j++) {
            kidx[j] = (int)rng.randrange(keys.size());
            pubs[j] = keys[kidx[j]].GetPubKey().Raw();
            if (rng.randrange(12) == 0) {
                pubs[j] = std::vector<unsigned char>(33, 0x11);
                pubs[j][0] = 0x05; // not a valid key encoding
                kidx[j] = -1;
            }
        }
        CScript spk;
        spk << m;
        for (const auto& p : pubs) spk << p;
        spk << n << OP_CHECKMULTISIG;
        const CMutableTransaction tx = SpendOf(spk);
        // signatures: usually for keys in list order (what passes), sometimes shuffled, corrupted,
        // signed by an unrelated key, or empty (empty ones keep the match eager)
        std::vector<int> order;
        for (int j = 0; j < n; j++) order.push_back(j);
        for (int j = n - 1; j > 0; j--) std::swap(order[j], order[rng.randrange(j + 1)]);
        std::vector<int> chosen(order.begin(), order.begin() + m);
        if (rng.randrange(4) != 0) std::sort(chosen.begin(), chosen.end());
        CScript sigs;
        sigs << OP_0;
        for (int c : chosen) {
            const int mode = (int)rng.randrange(20);
            const CKey& signer = (kidx[c] < 0 || mode == 0) ? keys[rng.randrange(keys.size())] : keys[kidx[c]];
            std::vector<unsigned char> sig = SignFor(signer, spk, tx, SIGHASH_ALL | SIGHASH_FORKID);
            if (mode == 1) sig[sig.size() - 3] ^= 0x01; // still DER, wrong signature
            if (mode == 2) sig.clear();
            if (mode == 3) sig = SignFor(signer, spk, tx, SIGHASH_ALL | SIGHASH_FORKID | SIGHASH_ANYONECANPAY);
            sigs << sig;
        }
        CMutableTransaction mtx = tx;
        mtx.vin[0].scriptSig = sigs;
        const Outcome o = RunBoth(sigs, spk, mtx);
        if (o.eager != o.deferred) {
            test::RecordFailure(strprintf("trial %d: %d-of-%d eager=%d deferred=%d", trial, m, n, o.eager, o.deferred),
                                __FILE__, __LINE__);
            return;
        }
        deferredRuns += o.groups;
        (o.eager ? valid : invalid)++;
    }
    // the interesting cases all occurred
    CHECK(deferredRuns > 500);
    CHECK(valid > 200);
    CHECK(invalid > 200);
}

TEST_CASE(sigbatch_tests, greedy_replay_edges) {
    // EvalDeferredMultisig against hand-built pair tables (rows: signatures, columns: key offset)
    DeferredMultisig g;
    g.m = 2;
    g.n = 3;
    g.keyOk = 0x7;
    // width 2: sig0 x {k0,k1}, sig1 x {k1,k2}
    const uint8_t allOk[4] = {1, 1, 1, 1};
    CHECK(EvalDeferredMultisig(g, allOk));
    const uint8_t skipFirstKey[4] = {0, 1, 0, 1}; // sig0 matches k1, sig1 matches k2
    CHECK(EvalDeferredMultisig(g, skipFirstKey));
    const uint8_t outOfOrder[4] = {0, 0, 1, 0}; // sig0 matches nothing reachable
    CHECK(!EvalDeferredMultisig(g, outOfOrder));
    const uint8_t sig1Only01[4] = {1, 0, 0, 0}; // sig0=k0, sig1 must be k1 or k2: neither
    CHECK(!EvalDeferredMultisig(g, sig1Only01));
    // a bad key is an error only if the match reaches it
    g.keyOk = 0x3; // k2 bad
    const uint8_t firstTwo[4] = {1, 0, 1, 0}; // sig0=k0, sig1=k1: k2 never visited
    CHECK(EvalDeferredMultisig(g, firstTwo));
    const uint8_t needsK2[4] = {1, 0, 0, 1}; // sig1 would match k2, but k2 is visited first as bad
    CHECK(!EvalDeferredMultisig(g, needsK2));
    g.keyOk = 0x6; // k0 bad: visited first
    CHECK(!EvalDeferredMultisig(g, allOk));
}

TEST_CASE(sigbatch_tests, checksig_deferral_matches_eager) {
    test::BasicTestingSetup setup("main");
    FastRandomContext rng(true);
    std::vector<CKey> keys(6);
    for (size_t i = 0; i < keys.size(); i++) keys[i].MakeNewKey(i % 2 == 0);
    int deferred = 0;
    for (int trial = 0; trial < 600; trial++) {
        const CKey& owner = keys[rng.randrange(keys.size())];
        // P2PK, CHECKSIGVERIFY chains and a CHECKSIG whose result is NOTed (fails under NULLFAIL
        // unless the signature is empty)
        const int shape = (int)rng.randrange(3);
        CScript spk;
        if (shape == 0) spk << owner.GetPubKey().Raw() << OP_CHECKSIG;
        else if (shape == 1) spk << owner.GetPubKey().Raw() << OP_CHECKSIGVERIFY << OP_TRUE;
        else spk << owner.GetPubKey().Raw() << OP_CHECKSIG << OP_NOT;
        const CMutableTransaction tx = SpendOf(spk);
        std::vector<unsigned char> sig = SignFor(rng.randrange(4) ? owner : keys[rng.randrange(keys.size())], spk, tx,
                                                 SIGHASH_ALL | SIGHASH_FORKID);
        const int mode = (int)rng.randrange(6);
        if (mode == 0) sig[sig.size() - 3] ^= 0x01;
        if (mode == 1) sig.clear();
        CScript ss;
        ss << sig;
        CMutableTransaction mtx = tx;
        mtx.vin[0].scriptSig = ss;
        const Outcome o = RunBoth(ss, spk, mtx);
        if (o.eager != o.deferred) {
            test::RecordFailure(strprintf("trial %d shape %d mode %d: eager=%d deferred=%d", trial, shape, mode, o.eager,
                                          o.deferred),
                                __FILE__, __LINE__);
            return;
        }
        deferred += o.checks > 0;
    }
    CHECK(deferred > 300);
}

// Deferral is bounded: a CHECKMULTISIG whose candidate pairs m*(n-m+1) exceed 2n (10-of-20: 110
// pairs against the 20 the reference's greedy loop can verify) runs eagerly, so a block at the
// sigop limit made of such spends costs no more than twice the reference's worst case. Typical
// shapes (2-of-3, 3-of-5, n-of-n) still defer. Verdicts match the eager run either way.
TEST_CASE(sigbatch_tests, multisig_deferral_is_bounded) {
    test::BasicTestingSetup setup("main");
    std::vector<CKey> keys(20);
    for (size_t i = 0; i < keys.size(); i++) keys[i].MakeNewKey(true);
    struct Shape { int m, n; bool defers; };
    for (const Shape sh : {Shape{10, 20, false}, Shape{5, 10, false}, Shape{2, 3, true}, Shape{3, 5, true},
                           Shape{20, 20, true}, Shape{1, 20, true}}) {
        CScript spk;
        spk << sh.m;
        for (int j = 0; j < sh.n; j++) spk << keys[j].GetPubKey().Raw();
        spk << sh.n << OP_CHECKMULTISIG;
        const CMutableTransaction tx = SpendOf(spk);
        CScript sigs;
        sigs << OP_0;
        for (int j = 0; j < sh.m; j++) sigs << SignFor(keys[2 * j * sh.n / (2 * sh.m)], spk, tx, SIGHASH_ALL | SIGHASH_FORKID);
        CMutableTransaction mtx = tx;
        mtx.vin[0].scriptSig = sigs;
        const Outcome o = RunBoth(sigs, spk, mtx);
        CHECK(o.eager && o.deferred);
        CHECK_EQ(o.groups, sh.defers ? 1u : 0u);
        // pairs queued for the batch: at most 2n
        CHECK(o.checks <= (size_t)(2 * sh.n));
    }
}
