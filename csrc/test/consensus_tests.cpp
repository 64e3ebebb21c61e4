// Consensus unit suites.
// Parity:
//   script_antireplay_tests  reference src/test/script_antireplay_tests.cpp (CScript::IsCommitment,
//                            ContextualCheckTransaction's OP_RETURN anti-replay window
//                            [BCPHeight, antiReplayOpReturnSunsetHeight], 'bad-txn-replay')
//   sigopcount_tests         reference src/test/sigopcount_tests.cpp (legacy / accurate / P2SH
//                            sigop counts, GetTransactionSigOpCount, the per-MB block limit and the
//                            per-transaction limit 'bad-txn-sigops')
#include "test/unittest.h"

#include "consensus/params.h"
#include "consensus/tx_verify.h"
#include "consensus/validation_state.h"
#include "node/coins.h"
#include "node/validation.h"
#include "script/interpreter.h"
#include "script/standard.h"

#include <limits>

using namespace bcp;
using namespace bcp::test;

static std::vector<unsigned char> Bytes(const CScript& s) { return std::vector<unsigned char>(s.begin(), s.end()); }
static std::vector<unsigned char> Bytes(const uint160& h) { return std::vector<unsigned char>(h.begin(), h.end()); }

// ------------------------------------------------------------------ script_antireplay_tests

TEST_CASE(script_antireplay_tests, is_commitment) {
    BasicTestingSetup setup;
    std::vector<unsigned char> data;
    CScript s = CScript() << OP_RETURN << data;
    CHECK(s.IsCommitment(data)); // empty commitment
    data.push_back(42);
    CHECK(!s.IsCommitment(data)); // wrong size
    s = CScript() << data;
    CHECK(!s.IsCommitment(data)); // not OP_RETURN
    s = CScript() << OP_RETURN << data;
    CHECK(s.IsCommitment(data));
    data[0] = 0x42;
    CHECK(!s.IsCommitment(data)); // wrong value
    const std::string str = "Bitcoin: A peer-to-peer Electronic Cash System";
    data.assign(str.begin(), str.end());
    CHECK(!s.IsCommitment(data));
    s = CScript() << OP_RETURN << data;
    CHECK(s.IsCommitment(data));
    data.resize(64); // 64-byte commitment still valid
    s = CScript() << OP_RETURN << data;
    CHECK(s.IsCommitment(data));
    data.push_back(23); // too large
    s = CScript() << OP_RETURN << data;
    CHECK(!s.IsCommitment(data));
    const Consensus::Params& p = Params().GetConsensus();
    s = CScript() << OP_RETURN << p.antiReplayOpReturnCommitment;
    CHECK(s.IsCommitment(p.antiReplayOpReturnCommitment));
}

TEST_CASE(script_antireplay_tests, antireplay_window) {
    TestingSetup setup("main");
    Chainstate& cs = *setup.node->chainstate;
    const Consensus::Params& p = cs.Params().GetConsensus();
    const int forkHeight = p.BCPHeight, sunset = p.antiReplayOpReturnSunsetHeight;
    REQUIRE(forkHeight < sunset);
    const int64_t t = 123456;
    CMutableTransaction mtx;
    mtx.nVersion = 1;
    mtx.vin.resize(1);
    mtx.vin[0].prevout = COutPoint(GetRandHash(), 0);
    mtx.vout.resize(1);
    mtx.vout[0].nValue = 1;
    auto check = [&](int height) {
        CValidationState st;
        const bool ok = cs.ContextualCheckTransaction(CTransaction(mtx), st, height, t);
        return std::make_pair(ok, st.GetRejectReason());
    };
    CHECK(check(sunset).first);
    CHECK(check(sunset + 1).first);
    CHECK(check(forkHeight - 1).first);
    mtx.vout[0].scriptPubKey = CScript() << OP_RETURN << OP_0; // wrong commitment: valid
    CHECK(check(sunset).first);
    mtx.vout[0].scriptPubKey = CScript() << OP_RETURN << p.antiReplayOpReturnCommitment;
    auto r = check(forkHeight);
    CHECK(!r.first);
    CHECK_EQ(r.second, std::string("bad-txn-replay"));
    r = check(sunset);
    CHECK(!r.first);
    CHECK_EQ(r.second, std::string("bad-txn-replay"));
    CHECK(check(forkHeight - 1).first); // before the fork
    CHECK(check(sunset + 1).first);     // after the sunset
    // the commitment in a second output is caught too
    mtx.vout.insert(mtx.vout.begin(), CTxOut(1, CScript() << OP_TRUE));
    CHECK(!check(forkHeight + 1).first);
}

// ------------------------------------------------------------------ sigopcount_tests

TEST_CASE(sigopcount_tests, GetSigOpCount) {
    BasicTestingSetup setup;
    CScript s1;
    CHECK_EQ(s1.GetSigOpCount(false), 0u);
    CHECK_EQ(s1.GetSigOpCount(true), 0u);
    uint160 dummy;
    s1 << OP_1 << Bytes(dummy) << Bytes(dummy) << OP_2 << OP_CHECKMULTISIG;
    CHECK_EQ(s1.GetSigOpCount(true), 2u);
    s1 << OP_IF << OP_CHECKSIG << OP_ENDIF;
    CHECK_EQ(s1.GetSigOpCount(true), 3u);
    CHECK_EQ(s1.GetSigOpCount(false), 21u);

    CScript p2sh = GetScriptForDestination(CScriptID(s1));
    CScript scriptSig;
    scriptSig << OP_0 << Bytes(s1);
    CHECK_EQ(p2sh.GetSigOpCount(scriptSig), 3u);

    std::vector<CPubKey> keys;
    for (int i = 0; i < 3; i++) {
        CKey k;
        k.MakeNewKey(true);
        keys.push_back(k.GetPubKey());
    }
    CScript s2 = GetScriptForMultisig(1, keys);
    CHECK_EQ(s2.GetSigOpCount(true), 3u);
    CHECK_EQ(s2.GetSigOpCount(false), 20u);
    p2sh = GetScriptForDestination(CScriptID(s2));
    CHECK_EQ(p2sh.GetSigOpCount(true), 0u);
    CHECK_EQ(p2sh.GetSigOpCount(false), 0u);
    CScript scriptSig2;
    scriptSig2 << OP_1 << Bytes(dummy) << Bytes(dummy) << Bytes(s2);
    CHECK_EQ(p2sh.GetSigOpCount(scriptSig2), 3u);
}

static ScriptError VerifyWithFlag(const CTransaction& output, const CMutableTransaction& input, uint32_t flags) {
    ScriptError error = SCRIPT_ERR_OK;
    const CTransaction in(input);
    const bool ret = VerifyScript(in.vin[0].scriptSig, output.vout[0].scriptPubKey, flags,
                                  TransactionSignatureChecker(&in, 0, output.vout[0].nValue), &error);
    CHECK((ret == true) == (error == SCRIPT_ERR_OK));
    return error;
}

static void BuildTxs(CMutableTransaction& spendingTx, CCoinsViewCache& coins, CMutableTransaction& creationTx,
                     const CScript& scriptPubKey, const CScript& scriptSig) {
    creationTx = CMutableTransaction();
    creationTx.nVersion = 1;
    creationTx.vin.resize(1);
    creationTx.vin[0].prevout.SetNull();
    creationTx.vout.resize(1);
    creationTx.vout[0].nValue = 1;
    creationTx.vout[0].scriptPubKey = scriptPubKey;
    spendingTx = CMutableTransaction();
    spendingTx.nVersion = 1;
    spendingTx.vin.resize(1);
    spendingTx.vin[0].prevout = COutPoint(creationTx.GetId(), 0);
    spendingTx.vin[0].scriptSig = scriptSig;
    spendingTx.vout.resize(1);
    spendingTx.vout[0].nValue = 1;
    AddCoins(coins, CTransaction(creationTx), 0);
}

TEST_CASE(sigopcount_tests, GetTxSigOpCost) {
    BasicTestingSetup setup;
    CMutableTransaction creationTx, spendingTx;
    CCoinsView dummy;
    CCoinsViewCache coins(&dummy);
    CKey key;
    key.MakeNewKey(true);
    const std::vector<unsigned char> pub = key.GetPubKey().Raw();
    const int flags = SCRIPT_VERIFY_P2SH;
    {
        CScript spk = CScript() << 1 << pub << pub << 2 << OP_CHECKMULTISIGVERIFY;
        BuildTxs(spendingTx, coins, creationTx, spk, CScript() << OP_0 << OP_0);
        CHECK_EQ(GetTransactionSigOpCount(CTransaction(spendingTx), coins, flags), 0u);
        CHECK_EQ(GetTransactionSigOpCount(CTransaction(creationTx), coins, flags), (uint64_t)MAX_PUBKEYS_PER_MULTISIG);
        CHECK(VerifyWithFlag(CTransaction(creationTx), spendingTx, flags) == SCRIPT_ERR_CHECKMULTISIGVERIFY);
    }
    {
        CScript redeem = CScript() << 1 << pub << pub << 2 << OP_CHECKMULTISIGVERIFY;
        CScript spk = GetScriptForDestination(CScriptID(redeem));
        BuildTxs(spendingTx, coins, creationTx, spk, CScript() << OP_0 << OP_0 << Bytes(redeem));
        CHECK_EQ(GetTransactionSigOpCount(CTransaction(spendingTx), coins, flags), 2u);
        CHECK(VerifyWithFlag(CTransaction(creationTx), spendingTx, flags) == SCRIPT_ERR_CHECKMULTISIGVERIFY);
    }
}

TEST_CASE(sigopcount_tests, consensus_sigops_limit) {
    CHECK_EQ(GetMaxBlockSigOpsCount(1), MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(123456), MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(1000000), MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(1000001), 2 * MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(1348592), 2 * MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(2000000), 2 * MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(2000001), 3 * MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(2654321), 3 * MAX_BLOCK_SIGOPS_PER_MB);
    CHECK_EQ(GetMaxBlockSigOpsCount(std::numeric_limits<uint32_t>::max()), 4295 * MAX_BLOCK_SIGOPS_PER_MB);
}

TEST_CASE(sigopcount_tests, max_sigops_per_tx) {
    CMutableTransaction tx;
    tx.nVersion = 1;
    tx.vin.resize(1);
    tx.vin[0].prevout = COutPoint(GetRandHash(), 0);
    tx.vout.resize(1);
    tx.vout[0].nValue = 1;
    {
        CValidationState st;
        CHECK(CheckRegularTransaction(CTransaction(tx), st, false));
    }
    for (size_t i = 0; i < MAX_TX_SIGOPS_COUNT; i++) tx.vout[0].scriptPubKey << OP_CHECKSIG;
    {
        CValidationState st;
        CHECK(CheckRegularTransaction(CTransaction(tx), st, false));
    }
    tx.vout[0].scriptPubKey << OP_CHECKSIG;
    {
        CValidationState st;
        CHECK(!CheckRegularTransaction(CTransaction(tx), st, false));
        CHECK_EQ(st.GetRejectReason(), std::string("bad-txn-sigops"));
    }
}
