// multisig_tests: bare CHECKMULTISIG scripts (2-of-2, 1-of-2, 2-of-3 escrow) - verification
// with every key combination and the exact script errors, standardness of well-formed and
// malformed multisig scripts, Solver / ExtractDestination(s) / IsMine, and SignSignature.
// Parity: reference src/test/multisig_tests.cpp (multisig_verify, multisig_IsStandard,
// multisig_Solver1, multisig_Sign).
#include "test/unittest.h"

#include "node/policy.h"
#include "script/interpreter.h"
#include "script/sign.h"
#include "script/standard.h"
#include "wallet/wallet.h"

using namespace bcp;

namespace {

std::vector<unsigned char> Bytes(const CPubKey& k) { return std::vector<unsigned char>(k.begin(), k.end()); }
std::vector<unsigned char> Bytes(const CKeyID& id) { return std::vector<unsigned char>(id.begin(), id.end()); }

// OP_0 <sig>... over SIGHASH_ALL (legacy digest, amount 0), as the reference's sign_multisig
CScript SignMultisig(const CScript& spk, const std::vector<CKey>& keys, const CMutableTransaction& tx, unsigned nIn) {
    const uint256 h = SignatureHash(spk, CTransaction(tx), nIn, SIGHASH_ALL, 0);
    CScript s;
    s << OP_0;
    for (const CKey& k : keys) {
        std::vector<unsigned char> sig;
        CHECK(k.Sign(h, sig));
        sig.push_back((unsigned char)SIGHASH_ALL);
        s << sig;
    }
    return s;
}

struct Fixture {
    CKey key[4];
    CScript a_and_b, a_or_b, escrow;
    CMutableTransaction from, to[3];
    Fixture() {
        for (CKey& k : key) k.MakeNewKey(true);
        a_and_b << OP_2 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << OP_2 << OP_CHECKMULTISIG;
        a_or_b << OP_1 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << OP_2 << OP_CHECKMULTISIG;
        escrow << OP_2 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << Bytes(key[2].GetPubKey()) << OP_3
               << OP_CHECKMULTISIG;
        from.vout.resize(3);
        from.vout[0].scriptPubKey = a_and_b;
        from.vout[1].scriptPubKey = a_or_b;
        from.vout[2].scriptPubKey = escrow;
        const uint256 fromId = CTransaction(from).GetHash();
        for (int i = 0; i < 3; i++) {
            to[i].vin.resize(1);
            to[i].vout.resize(1);
            to[i].vin[0].prevout = COutPoint(fromId, (uint32_t)i);
            to[i].vout[0].nValue = 1;
        }
    }
};

} // namespace

TEST_CASE(multisig_tests, multisig_verify) {
    Fixture f;
    const uint32_t flags = SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_STRICTENC;
    auto verify = [&](const CScript& sig, const CScript& spk, int txi, ScriptError& err) {
        return VerifyScript(sig, spk, flags, MutableTransactionSignatureChecker(&f.to[txi], 0, 0), &err);
    };
    ScriptError err;
    // a AND b
    CHECK(verify(SignMultisig(f.a_and_b, {f.key[0], f.key[1]}, f.to[0], 0), f.a_and_b, 0, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
    for (int i = 0; i < 4; i++) {
        CHECK(!verify(SignMultisig(f.a_and_b, {f.key[i]}, f.to[0], 0), f.a_and_b, 0, err));
        CHECK_EQ((int)err, (int)SCRIPT_ERR_INVALID_STACK_OPERATION);
        CHECK(!verify(SignMultisig(f.a_and_b, {f.key[1], f.key[i]}, f.to[0], 0), f.a_and_b, 0, err));
        CHECK_EQ((int)err, (int)SCRIPT_ERR_EVAL_FALSE);
    }
    // a OR b
    for (int i = 0; i < 4; i++) {
        const bool ok = verify(SignMultisig(f.a_or_b, {f.key[i]}, f.to[1], 0), f.a_or_b, 1, err);
        if (i < 2) {
            CHECK(ok);
            CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
        } else {
            CHECK(!ok);
            CHECK_EQ((int)err, (int)SCRIPT_ERR_EVAL_FALSE);
        }
    }
    CScript junk;
    junk << OP_0 << OP_1; // a "signature" that is not DER
    CHECK(!verify(junk, f.a_or_b, 1, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_SIG_DER);
    // 2-of-3 escrow: signatures must come in key order
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            const bool ok = verify(SignMultisig(f.escrow, {f.key[i], f.key[j]}, f.to[2], 0), f.escrow, 2, err);
            if (i < j && j < 3) {
                CHECK(ok);
                CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
            } else {
                CHECK(!ok);
                CHECK_EQ((int)err, (int)SCRIPT_ERR_EVAL_FALSE);
            }
        }
}

TEST_CASE(multisig_tests, multisig_IsStandard) {
    Fixture f;
    txnouttype t;
    CHECK(IsStandard(f.a_and_b, t));
    CHECK(IsStandard(f.a_or_b, t));
    CHECK(IsStandard(f.escrow, t));
    CScript one_of_four;
    one_of_four << OP_1;
    for (int i = 0; i < 4; i++) one_of_four << Bytes(f.key[i].GetPubKey());
    one_of_four << OP_4 << OP_CHECKMULTISIG;
    CHECK(!IsStandard(one_of_four, t)); // bare multisig is limited to 3 keys
    const auto k0 = Bytes(f.key[0].GetPubKey()), k1 = Bytes(f.key[1].GetPubKey());
    CScript bad[6];
    bad[0] << OP_3 << k0 << k1 << OP_2 << OP_CHECKMULTISIG; // m > n
    bad[1] << OP_2 << k0 << k1 << OP_3 << OP_CHECKMULTISIG; // n != number of keys
    bad[2] << OP_0 << k0 << k1 << OP_2 << OP_CHECKMULTISIG; // m = 0
    bad[3] << OP_1 << k0 << k1 << OP_0 << OP_CHECKMULTISIG; // n = 0
    bad[4] << OP_1 << k0 << k1 << OP_CHECKMULTISIG;         // no n
    bad[5] << OP_1 << k0 << k1;                             // no CHECKMULTISIG
    for (const CScript& s : bad) CHECK(!IsStandard(s, t));
}

TEST_CASE(multisig_tests, multisig_Solver1) {
    CBasicKeyStore keystore, empty, partial;
    CKey key[3];
    CTxDestination addr[3];
    for (int i = 0; i < 3; i++) {
        key[i].MakeNewKey(true);
        keystore.AddKey(key[i]);
        addr[i] = CTxDestination(key[i].GetPubKey().GetID());
    }
    partial.AddKey(key[0]);
    std::vector<std::vector<unsigned char>> sol;
    txnouttype t;
    {
        CScript s;
        s << Bytes(key[0].GetPubKey()) << OP_CHECKSIG;
        CHECK(Solver(s, t, sol));
        CHECK_EQ(sol.size(), (size_t)1);
        CTxDestination d;
        CHECK(ExtractDestination(s, d));
        CHECK(d == addr[0]);
        CHECK(IsMine(keystore, s) != ISMINE_NO);
        CHECK(IsMine(empty, s) == ISMINE_NO);
    }
    {
        CScript s;
        s << OP_DUP << OP_HASH160 << Bytes(key[0].GetPubKey().GetID()) << OP_EQUALVERIFY << OP_CHECKSIG;
        CHECK(Solver(s, t, sol));
        CHECK_EQ(sol.size(), (size_t)1);
        CTxDestination d;
        CHECK(ExtractDestination(s, d));
        CHECK(d == addr[0]);
        CHECK(IsMine(keystore, s) != ISMINE_NO);
        CHECK(IsMine(empty, s) == ISMINE_NO);
    }
    {
        CScript s;
        s << OP_2 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << OP_2 << OP_CHECKMULTISIG;
        CHECK(Solver(s, t, sol));
        CHECK_EQ(sol.size(), (size_t)4); // m, two keys, n
        CTxDestination d;
        CHECK(!ExtractDestination(s, d));
        CHECK(IsMine(keystore, s) != ISMINE_NO);
        CHECK(IsMine(empty, s) == ISMINE_NO);
        CHECK(IsMine(partial, s) == ISMINE_NO);
    }
    {
        CScript s;
        s << OP_1 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << OP_2 << OP_CHECKMULTISIG;
        CHECK(Solver(s, t, sol));
        CHECK_EQ(sol.size(), (size_t)4);
        std::vector<CTxDestination> ds;
        int nReq = 0;
        CHECK(ExtractDestinations(s, t, ds, nReq));
        CHECK(ds.size() == 2 && ds[0] == addr[0] && ds[1] == addr[1]);
        CHECK_EQ(nReq, 1);
        CHECK(IsMine(keystore, s) != ISMINE_NO);
        CHECK(IsMine(empty, s) == ISMINE_NO);
        CHECK(IsMine(partial, s) == ISMINE_NO);
    }
    {
        CScript s;
        s << OP_2 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << Bytes(key[2].GetPubKey()) << OP_3
          << OP_CHECKMULTISIG;
        CHECK(Solver(s, t, sol));
        CHECK_EQ(sol.size(), (size_t)5);
    }
}

TEST_CASE(multisig_tests, multisig_Sign) {
    Fixture f;
    CBasicKeyStore keystore;
    for (const CKey& k : f.key) keystore.AddKey(k);
    const CScript spks[3] = {f.a_and_b, f.a_or_b, f.escrow};
    for (int i = 0; i < 3; i++) {
        CHECK(SignSignature(keystore, spks[i], f.to[i], 0, 0, SIGHASH_ALL | SIGHASH_FORKID));
        // and the result verifies under the FORKID rules
        ScriptError err;
        CHECK(VerifyScript(f.to[i].vin[0].scriptSig, spks[i],
                           SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_STRICTENC | SCRIPT_ENABLE_SIGHASH_FORKID,
                           MutableTransactionSignatureChecker(&f.to[i], 0, 0), &err));
        CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
    }
}
