// script_P2SH_tests: pay-to-script-hash signing and verification over every combination of
// keys and straight/P2SH, pubkey/pubkeyhash outputs; only the outer P2SH layer evaluates its
// redeem script; CScript::IsPayToScriptHash on exact and look-alike encodings; the switch-over
// (a P2SH output is a plain hash check without SCRIPT_VERIFY_P2SH); multisig redeem scripts;
// AreInputsStandard and GetP2SHSigOpCount at and over MAX_P2SH_SIGOPS.
// Parity: reference src/test/script_P2SH_tests.cpp (sign, norecurse, set, is, switchover,
// AreInputsStandard).
#include "test/unittest.h"

#include "consensus/tx_verify.h"
#include "node/coins.h"
#include "node/policy.h"
#include "script/interpreter.h"
#include "script/sign.h"
#include "script/standard.h"
#include "wallet/wallet.h"

using namespace bcp;
using bcp::test::BasicTestingSetup;

namespace {

std::vector<unsigned char> Ser(const CScript& s) { return std::vector<unsigned char>(s.begin(), s.end()); }
std::vector<unsigned char> Bytes(const CPubKey& k) { return std::vector<unsigned char>(k.begin(), k.end()); }

// dummy funding and spending transactions around one input (reference Verify helper)
bool Verify(const CScript& scriptSig, const CScript& scriptPubKey, bool fStrict, ScriptError& err) {
    CMutableTransaction txFrom;
    txFrom.vout.resize(1);
    txFrom.vout[0].scriptPubKey = scriptPubKey;
    CMutableTransaction txTo;
    txTo.vin.resize(1);
    txTo.vout.resize(1);
    txTo.vin[0].prevout = COutPoint(txFrom.GetId(), 0);
    txTo.vin[0].scriptSig = scriptSig;
    txTo.vout[0].nValue = 1;
    return VerifyScript(scriptSig, scriptPubKey,
                        (fStrict ? SCRIPT_VERIFY_P2SH : SCRIPT_VERIFY_NONE) | SCRIPT_ENABLE_SIGHASH_FORKID,
                        MutableTransactionSignatureChecker(&txTo, 0, txFrom.vout[0].nValue), &err);
}

} // namespace

TEST_CASE(script_P2SH_tests, sign) {
    BasicTestingSetup setup;
    CBasicKeyStore keystore;
    CKey key[4];
    for (CKey& k : key) {
        k.MakeNewKey(true);
        keystore.AddKey(k);
    }
    // 8 scripts: different keys, straight / P2SH, pubkey / pubkeyhash
    CScript standard[4];
    standard[0] << Bytes(key[0].GetPubKey()) << OP_CHECKSIG;
    standard[1] = GetScriptForDestination(key[1].GetPubKey().GetID());
    standard[2] << Bytes(key[1].GetPubKey()) << OP_CHECKSIG;
    standard[3] = GetScriptForDestination(key[2].GetPubKey().GetID());
    CScript eval[4];
    for (int i = 0; i < 4; i++) {
        keystore.AddCScript(standard[i]);
        eval[i] = GetScriptForDestination(CScriptID(standard[i]));
    }
    CMutableTransaction txFrom;
    txFrom.vout.resize(8);
    for (int i = 0; i < 4; i++) {
        txFrom.vout[i] = CTxOut(COIN, eval[i]);
        txFrom.vout[i + 4] = CTxOut(COIN, standard[i]);
    }
    std::string reason;
    CHECK(IsStandardTx(CTransaction(txFrom), reason));

    CMutableTransaction txTo[8];
    for (int i = 0; i < 8; i++) {
        txTo[i].vin.resize(1);
        txTo[i].vout.resize(1);
        txTo[i].vin[0].prevout = COutPoint(txFrom.GetId(), (uint32_t)i);
        txTo[i].vout[0].nValue = 1;
        CHECK(IsMine(keystore, txFrom.vout[i].scriptPubKey) != ISMINE_NO);
    }
    for (int i = 0; i < 8; i++)
        CHECK(SignSignature(keystore, txFrom.vout[i].scriptPubKey, txTo[i], 0, txFrom.vout[i].nValue,
                            SIGHASH_ALL | SIGHASH_FORKID));
    // every scriptSig verifies only against its own output
    for (int i = 0; i < 8; i++) {
        for (int j = 0; j < 8; j++) {
            const CScript save = txTo[i].vin[0].scriptSig;
            txTo[i].vin[0].scriptSig = txTo[j].vin[0].scriptSig;
            const CTxOut& out = txFrom.vout[txTo[i].vin[0].prevout.n];
            ScriptError err;
            const bool ok = VerifyScript(txTo[i].vin[0].scriptSig, out.scriptPubKey,
                                         SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_STRICTENC | SCRIPT_ENABLE_SIGHASH_FORKID,
                                         MutableTransactionSignatureChecker(&txTo[i], 0, out.nValue), &err);
            CHECK_EQ(ok, i == j);
            txTo[i].vin[0].scriptSig = save;
        }
    }
}

TEST_CASE(script_P2SH_tests, norecurse) {
    ScriptError err;
    CScript invalidAsScript;
    invalidAsScript << OP_INVALIDOPCODE << OP_INVALIDOPCODE;
    const CScript p2sh = GetScriptForDestination(CScriptID(invalidAsScript));
    CScript scriptSig;
    scriptSig << Ser(invalidAsScript);
    // the redeem script runs and hits OP_INVALIDOPCODE
    CHECK(!Verify(scriptSig, p2sh, true, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_BAD_OPCODE);
    // a P2SH script used as a redeem script is only a hash check: no second evaluation
    const CScript p2sh2 = GetScriptForDestination(CScriptID(p2sh));
    CScript scriptSig2;
    scriptSig2 << Ser(invalidAsScript) << Ser(p2sh);
    CHECK(Verify(scriptSig2, p2sh2, true, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
}

TEST_CASE(script_P2SH_tests, set) {
    BasicTestingSetup setup;
    CBasicKeyStore keystore;
    CKey key[4];
    std::vector<CPubKey> keys;
    for (CKey& k : key) {
        k.MakeNewKey(true);
        keystore.AddKey(k);
        keys.push_back(k.GetPubKey());
    }
    CScript inner[4];
    inner[0] = GetScriptForDestination(key[0].GetPubKey().GetID());
    inner[1] = GetScriptForMultisig(2, std::vector<CPubKey>(keys.begin(), keys.begin() + 2));
    inner[2] = GetScriptForMultisig(1, std::vector<CPubKey>(keys.begin(), keys.begin() + 2));
    inner[3] = GetScriptForMultisig(2, std::vector<CPubKey>(keys.begin(), keys.begin() + 3));
    CScript outer[4];
    for (int i = 0; i < 4; i++) {
        outer[i] = GetScriptForDestination(CScriptID(inner[i]));
        keystore.AddCScript(inner[i]);
    }
    CMutableTransaction txFrom;
    txFrom.vout.resize(4);
    for (int i = 0; i < 4; i++) txFrom.vout[i] = CTxOut(CENT, outer[i]);
    std::string reason;
    CHECK(IsStandardTx(CTransaction(txFrom), reason));
    CMutableTransaction txTo[4];
    for (int i = 0; i < 4; i++) {
        txTo[i].vin.resize(1);
        txTo[i].vout.resize(1);
        txTo[i].vin[0].prevout = COutPoint(txFrom.GetId(), (uint32_t)i);
        txTo[i].vout[0] = CTxOut(CENT, inner[i]);
        CHECK(IsMine(keystore, txFrom.vout[i].scriptPubKey) != ISMINE_NO);
    }
    for (int i = 0; i < 4; i++) {
        CHECK(SignSignature(keystore, txFrom.vout[i].scriptPubKey, txTo[i], 0, CENT, SIGHASH_ALL | SIGHASH_FORKID));
        CHECK(IsStandardTx(CTransaction(txTo[i]), reason));
    }
}

TEST_CASE(script_P2SH_tests, is) {
    uint160 dummy;
    const std::vector<unsigned char> d(dummy.begin(), dummy.end());
    CScript p2sh;
    p2sh << OP_HASH160 << d << OP_EQUAL;
    CHECK(p2sh.IsPayToScriptHash());

    std::vector<unsigned char> direct = {OP_HASH160, 20};
    direct.resize(22, 0);
    direct.push_back(OP_EQUAL);
    CHECK(CScript(direct.begin(), direct.end()).IsPayToScriptHash());
    // the same 20 bytes behind OP_PUSHDATA1/2/4 is not P2SH
    std::vector<unsigned char> pd1 = {OP_HASH160, OP_PUSHDATA1, 20};
    pd1.resize(23, 0);
    pd1.push_back(OP_EQUAL);
    CHECK(!CScript(pd1.begin(), pd1.end()).IsPayToScriptHash());
    std::vector<unsigned char> pd2 = {OP_HASH160, OP_PUSHDATA2, 20, 0};
    pd2.resize(24, 0);
    pd2.push_back(OP_EQUAL);
    CHECK(!CScript(pd2.begin(), pd2.end()).IsPayToScriptHash());
    std::vector<unsigned char> pd4 = {OP_HASH160, OP_PUSHDATA4, 20, 0, 0, 0};
    pd4.resize(26, 0);
    pd4.push_back(OP_EQUAL);
    CHECK(!CScript(pd4.begin(), pd4.end()).IsPayToScriptHash());

    CScript not_p2sh;
    CHECK(!not_p2sh.IsPayToScriptHash());
    not_p2sh.clear();
    not_p2sh << OP_HASH160 << d << d << OP_EQUAL;
    CHECK(!not_p2sh.IsPayToScriptHash());
    not_p2sh.clear();
    not_p2sh << OP_NOP << d << OP_EQUAL;
    CHECK(!not_p2sh.IsPayToScriptHash());
    not_p2sh.clear();
    not_p2sh << OP_HASH160 << d << OP_CHECKSIG;
    CHECK(!not_p2sh.IsPayToScriptHash());
}

TEST_CASE(script_P2SH_tests, switchover) {
    CScript notValid;
    notValid << OP_11 << OP_12 << OP_EQUALVERIFY;
    CScript scriptSig;
    scriptSig << Ser(notValid);
    const CScript fund = GetScriptForDestination(CScriptID(notValid));
    ScriptError err;
    // old rules: only the hash is checked
    CHECK(Verify(scriptSig, fund, false, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_OK);
    // P2SH rules: the redeem script runs and fails
    CHECK(!Verify(scriptSig, fund, true, err));
    CHECK_EQ((int)err, (int)SCRIPT_ERR_EQUALVERIFY);
}

TEST_CASE(script_P2SH_tests, AreInputsStandard) {
    BasicTestingSetup setup;
    CCoinsView coinsDummy;
    CCoinsViewCache coins(&coinsDummy);
    CBasicKeyStore keystore;
    CKey key[6];
    std::vector<CPubKey> keys;
    for (CKey& k : key) {
        k.MakeNewKey(true);
        keystore.AddKey(k);
    }
    for (int i = 0; i < 3; i++) keys.push_back(key[i].GetPubKey());

    CMutableTransaction txFrom;
    txFrom.vout.resize(7);
    const CScript pay1 = GetScriptForDestination(key[0].GetPubKey().GetID());
    keystore.AddCScript(pay1);
    const CScript pay1of3 = GetScriptForMultisig(1, keys);
    txFrom.vout[0] = CTxOut(1000, GetScriptForDestination(CScriptID(pay1))); // P2SH (CHECKSIG)
    txFrom.vout[1] = CTxOut(2000, pay1);                                     // plain CHECKSIG
    txFrom.vout[2] = CTxOut(3000, pay1of3);                                  // plain CHECKMULTISIG
    // 1-of-3 AND 2-of-3: non-standard bare, fine inside P2SH
    CScript oneAndTwo;
    oneAndTwo << OP_1 << Bytes(key[0].GetPubKey()) << Bytes(key[1].GetPubKey()) << Bytes(key[2].GetPubKey());
    oneAndTwo << OP_3 << OP_CHECKMULTISIGVERIFY;
    oneAndTwo << OP_2 << Bytes(key[3].GetPubKey()) << Bytes(key[4].GetPubKey()) << Bytes(key[5].GetPubKey());
    oneAndTwo << OP_3 << OP_CHECKMULTISIG;
    keystore.AddCScript(oneAndTwo);
    txFrom.vout[3] = CTxOut(4000, GetScriptForDestination(CScriptID(oneAndTwo)));
    // exactly MAX_P2SH_SIGOPS
    CScript fifteenSigops;
    fifteenSigops << OP_1;
    for (unsigned i = 0; i < MAX_P2SH_SIGOPS; i++) fifteenSigops << Bytes(key[i % 3].GetPubKey());
    fifteenSigops << OP_15 << OP_CHECKMULTISIG;
    keystore.AddCScript(fifteenSigops);
    txFrom.vout[4] = CTxOut(5000, GetScriptForDestination(CScriptID(fifteenSigops)));
    // over the limit (vout[5] pays fifteenSigops' hash, as in the reference)
    CScript sixteenSigops;
    sixteenSigops << OP_16 << OP_CHECKMULTISIG;
    keystore.AddCScript(sixteenSigops);
    txFrom.vout[5] = CTxOut(5000, GetScriptForDestination(CScriptID(fifteenSigops)));
    CScript twentySigops;
    twentySigops << OP_CHECKMULTISIG;
    keystore.AddCScript(twentySigops);
    txFrom.vout[6] = CTxOut(6000, GetScriptForDestination(CScriptID(twentySigops)));
    AddCoins(coins, CTransaction(txFrom), 0);

    CMutableTransaction txTo;
    txTo.vout.resize(1);
    txTo.vout[0].scriptPubKey = GetScriptForDestination(key[1].GetPubKey().GetID());
    txTo.vin.resize(5);
    for (int i = 0; i < 5; i++) txTo.vin[i].prevout = COutPoint(txFrom.GetId(), (uint32_t)i);
    for (int i = 0; i < 3; i++)
        CHECK(SignSignature(keystore, txFrom.vout[i].scriptPubKey, txTo, (unsigned)i, txFrom.vout[i].nValue,
                            SIGHASH_ALL | SIGHASH_FORKID));
    // not signable here; dummy signatures that carry the right redeem scripts
    txTo.vin[3].scriptSig << OP_11 << OP_11 << Ser(oneAndTwo);
    txTo.vin[4].scriptSig << Ser(fifteenSigops);
    CHECK(AreInputsStandard(CTransaction(txTo), coins));
    // 1 (vin[0]) + 6 (vin[3]) + 15 (vin[4])
    CHECK_EQ(GetP2SHSigOpCount(CTransaction(txTo), coins), (uint64_t)22);

    CMutableTransaction nonStd1;
    nonStd1.vout.resize(1);
    nonStd1.vout[0] = CTxOut(1000, GetScriptForDestination(key[1].GetPubKey().GetID()));
    nonStd1.vin.resize(1);
    nonStd1.vin[0].prevout = COutPoint(txFrom.GetId(), 5);
    nonStd1.vin[0].scriptSig << Ser(sixteenSigops);
    CHECK(!AreInputsStandard(CTransaction(nonStd1), coins));
    CHECK_EQ(GetP2SHSigOpCount(CTransaction(nonStd1), coins), (uint64_t)16);

    CMutableTransaction nonStd2;
    nonStd2.vout.resize(1);
    nonStd2.vout[0] = CTxOut(1000, GetScriptForDestination(key[1].GetPubKey().GetID()));
    nonStd2.vin.resize(1);
    nonStd2.vin[0].prevout = COutPoint(txFrom.GetId(), 6);
    nonStd2.vin[0].scriptSig << Ser(twentySigops);
    CHECK(!AreInputsStandard(CTransaction(nonStd2), coins));
    CHECK_EQ(GetP2SHSigOpCount(CTransaction(nonStd2), coins), (uint64_t)20);
}
