// sighash_recipe_tests: the device signature-hash recipe (K7) must reproduce SignatureHash bit for
// bit. Parity: reference src/script/interpreter.cpp:1354-1404 (FORKID digest) and
// src/test/sighash_tests.cpp (randomized transactions x hash types). A divergent digest would
// make the GPU-validated chain split from the reference's, so every case is exact: random
// transactions of 1-4 inputs and 0-4 outputs, every base hash type with and without
// ANYONECANPAY, script codes of 0-300 bytes, and the block path (DeferringSignatureChecker with
// recipes, CPU fallback evaluation) against eager verification.
#include "test/unittest.h"

#include "keys/key.h"
#include "node/sigverify.h"
#include "script/interpreter.h"
#include "script/script.h"
#include "script/sighash_recipe.h"
#include "script/standard.h"
#include "util/strencodings.h"

#include <cstring>

using namespace bcp;

namespace {

CMutableTransaction RandomTx(FastRandomContext& rng) {
    CMutableTransaction tx;
    tx.nVersion = (int32_t)rng.rand32();
    tx.nLockTime = rng.randrange(2) ? 0 : rng.rand32();
    const int nin = 1 + (int)rng.randrange(4), nout = (int)rng.randrange(5);
    for (int i = 0; i < nin; i++) {
        CTxIn in;
        in.prevout = COutPoint(rng.rand256(), rng.rand32());
        in.nSequence = rng.randrange(2) ? 0xffffffffu : rng.rand32();
        tx.vin.push_back(in);
    }
    for (int i = 0; i < nout; i++) {
        std::vector<unsigned char> spk(rng.randrange(40));
        for (auto& b : spk) b = (unsigned char)rng.randrange(256);
        tx.vout.push_back(CTxOut((Amount)rng.randrange(1000000000), CScript(spk.begin(), spk.end())));
    }
    return tx;
}

const uint32_t kHashTypes[] = {0x41, 0x42, 0x43, 0xc1, 0xc2, 0xc3, 0x40, 0x44, 0x5f, 0x01, 0x03};

} // namespace

TEST_CASE(sighash_recipe_tests, recipe_matches_signature_hash) {
    FastRandomContext rng(true);
    int viaRecipe = 0;
    for (int trial = 0; trial < 4000; trial++) {
        const CTransaction tx(RandomTx(rng));
        const PrecomputedTransactionData txdata(tx);
        const unsigned nIn = (unsigned)rng.randrange(tx.vin.size());
        const uint32_t ht = rng.randrange(8) ? kHashTypes[rng.randrange(sizeof(kHashTypes) / 4)] : rng.randrange(256);
        std::vector<unsigned char> code(rng.randrange(4) ? rng.randrange(32) : rng.randrange(300));
        for (auto& b : code) b = (unsigned char)rng.randrange(256);
        const CScript sc(code.begin(), code.end());
        const Amount amount = (Amount)rng.randrange(2100000000000000ULL);
        const uint32_t flags = rng.randrange(8) ? SCRIPT_ENABLE_SIGHASH_FORKID : 0u;
        gpu::SighashTx t;
        gpu::SighashJob j;
        FillSighashTx(tx, txdata, t);
        if (!FillSighashJob(tx, nIn, ht, amount, flags, 0, 0, (uint32_t)code.size(), j)) {
            // only legacy digests and SIGHASH_SINGLE with a matching output stay on the CPU
            const bool single = (ht & 0x1f) == SIGHASH_SINGLE && nIn < tx.vout.size();
            CHECK(!(ht & SIGHASH_FORKID) || !(flags & SCRIPT_ENABLE_SIGHASH_FORKID) || single);
            continue;
        }
        viaRecipe++;
        const uint256 want = SignatureHash(sc, tx, nIn, ht, amount, &txdata, flags);
        if (SighashFromRecipe(t, j, code.data()) != want) {
            test::RecordFailure(strprintf("trial %d: hash type %#x, %zu-byte code, input %u of %zu, %zu outputs", trial,
                                          ht, code.size(), nIn, tx.vin.size(), tx.vout.size()),
                                __FILE__, __LINE__);
            return;
        }
    }
    CHECK(viaRecipe > 2000);
}

// The block path: P2PKH spends (25-byte code: a recipe) and P2PK spends (35/67-byte code: a CPU
// digest) under every FORKID hash type, valid and corrupted, deferred with recipes and verified by
// the CPU batch path (DeferredDigest), against eager verification.
TEST_CASE(sighash_recipe_tests, recipe_deferral_matches_eager) {
    test::BasicTestingSetup setup("main");
    FastRandomContext rng(true);
    const uint32_t flags = STANDARD_SCRIPT_VERIFY_FLAGS;
    std::vector<CKey> keys(4);
    for (size_t i = 0; i < keys.size(); i++) keys[i].MakeNewKey(i % 2 == 0);
    int recipes = 0, agree = 0;
    for (int trial = 0; trial < 400; trial++) {
        const CKey& key = keys[rng.randrange(keys.size())];
        const bool p2pkh = rng.randrange(3) != 0;
        CScript spk;
        if (p2pkh) spk = GetScriptForDestination(key.GetPubKey().GetID());
        else spk << key.GetPubKey().Raw() << OP_CHECKSIG;
        CMutableTransaction mtx = RandomTx(rng);
        const unsigned nIn = (unsigned)rng.randrange(mtx.vin.size());
        const Amount amount = (Amount)rng.randrange(1000000000);
        const uint32_t ht = kHashTypes[rng.randrange(6)];
        const uint256 h = SignatureHash(spk, CTransaction(mtx), nIn, ht, amount, nullptr, flags);
        std::vector<unsigned char> sig;
        (rng.randrange(5) ? key : keys[rng.randrange(keys.size())]).Sign(h, sig);
        if (rng.randrange(6) == 0) sig[sig.size() - 2] ^= 0x01;
        sig.push_back((unsigned char)ht);
        CScript ss;
        ss << sig;
        if (p2pkh) ss << key.GetPubKey().Raw();
        mtx.vin[nIn].scriptSig = ss;
        const CTransaction tx(mtx);
        const PrecomputedTransactionData txdata(tx);
        TransactionSignatureChecker eager(&tx, nIn, amount, &txdata);
        const bool e = VerifyScript(ss, spk, flags, eager);
        std::vector<DeferredSigCheck> sink;
        DeferringSignatureChecker lazy(&tx, nIn, amount, &txdata, &sink);
        lazy.SetRecipes(true);
        bool d = VerifyScript(ss, spk, flags, lazy);
        for (const DeferredSigCheck& c : sink) recipes += c.recipe;
        if (d) d = BatchVerifySignatures(sink, nullptr, false, false, false);
        if (e != d) {
            test::RecordFailure(strprintf("trial %d: %s, hash type %#x: eager=%d deferred=%d", trial,
                                          p2pkh ? "P2PKH" : "P2PK", ht, e, d),
                                __FILE__, __LINE__);
            return;
        }
        agree += e;
    }
    CHECK(recipes > 150);
    CHECK(agree > 150);
}
