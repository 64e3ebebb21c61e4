#include "consensuslib/bitcoinconsensus.h"
#include "primitives/transaction.h"
#include "script/interpreter.h"

using namespace bcp;

static int SetError(bitcoinconsensus_error* ret, bitcoinconsensus_error serror) {
    if (ret) *ret = serror;
    return 0;
}

static bool FlagsValid(unsigned int flags) {
    return (flags & ~(bitcoinconsensus_SCRIPT_FLAGS_VERIFY_ALL | bitcoinconsensus_SCRIPT_ENABLE_SIGHASH_FORKID)) == 0;
}

static int VerifyScript(const uint8_t* scriptPubKey, unsigned int scriptPubKeyLen, Amount amount, const uint8_t* txTo,
                        unsigned int txToLen, unsigned int nIn, unsigned int flags, bitcoinconsensus_error* err) {
    if (!FlagsValid(flags)) return SetError(err, bitcoinconsensus_ERR_INVALID_FLAGS);
    try {
        SpanReader r(txTo, txToLen, SER_NETWORK, PROTOCOL_VERSION);
        CMutableTransaction mtx;
        r >> mtx;
        const CTransaction tx(mtx);
        if (nIn >= tx.vin.size()) return SetError(err, bitcoinconsensus_ERR_TX_INDEX);
        if (r.size() != 0 || GetSerializeSize(tx) != txToLen) return SetError(err, bitcoinconsensus_ERR_TX_SIZE_MISMATCH);
        SetError(err, bitcoinconsensus_ERR_OK);
        const PrecomputedTransactionData txdata(tx);
        const CScript spk(scriptPubKey, scriptPubKey + scriptPubKeyLen);
        return VerifyScript(tx.vin[nIn].scriptSig, spk, flags, TransactionSignatureChecker(&tx, nIn, amount, &txdata),
                            nullptr)
                   ? 1
                   : 0;
    } catch (const std::exception&) {
        return SetError(err, bitcoinconsensus_ERR_TX_DESERIALIZE);
    }
}

int bitcoinconsensus_verify_script_with_amount(const uint8_t* scriptPubKey, unsigned int scriptPubKeyLen,
                                               int64_t amount, const uint8_t* txTo, unsigned int txToLen,
                                               unsigned int nIn, unsigned int flags, bitcoinconsensus_error* err) {
    return VerifyScript(scriptPubKey, scriptPubKeyLen, amount, txTo, txToLen, nIn, flags, err);
}

int bitcoinconsensus_verify_script(const uint8_t* scriptPubKey, unsigned int scriptPubKeyLen, const uint8_t* txTo,
                                   unsigned int txToLen, unsigned int nIn, unsigned int flags,
                                   bitcoinconsensus_error* err) {
    if (flags & bitcoinconsensus_SCRIPT_ENABLE_SIGHASH_FORKID) return SetError(err, bitcoinconsensus_ERR_AMOUNT_REQUIRED);
    return VerifyScript(scriptPubKey, scriptPubKeyLen, 0, txTo, txToLen, nIn, flags, err);
}

unsigned int bitcoinconsensus_version() { return BITCOINCONSENSUS_API_VER; }
