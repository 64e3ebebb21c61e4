// libbcpconsensus: stable C API for script verification.
// Parity: reference src/script/bitcoinconsensus.{h,cpp} (API version 1, error codes,
// flag set incl. SCRIPT_ENABLE_SIGHASH_FORKID which requires the _with_amount call).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BITCOINCONSENSUS_API_VER 1

typedef enum bitcoinconsensus_error_t {
    bitcoinconsensus_ERR_OK = 0,
    bitcoinconsensus_ERR_TX_INDEX,
    bitcoinconsensus_ERR_TX_SIZE_MISMATCH,
    bitcoinconsensus_ERR_TX_DESERIALIZE,
    bitcoinconsensus_ERR_AMOUNT_REQUIRED,
    bitcoinconsensus_ERR_INVALID_FLAGS,
} bitcoinconsensus_error;

enum {
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NONE = 0,
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_P2SH = (1U << 0),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_DERSIG = (1U << 2),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NULLDUMMY = (1U << 4),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKLOCKTIMEVERIFY = (1U << 9),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKSEQUENCEVERIFY = (1U << 10),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_WITNESS_DEPRECATED = (1U << 11),
    bitcoinconsensus_SCRIPT_ENABLE_SIGHASH_FORKID = (1U << 16),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_ALL =
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_P2SH | bitcoinconsensus_SCRIPT_FLAGS_VERIFY_DERSIG |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NULLDUMMY | bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKLOCKTIMEVERIFY |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKSEQUENCEVERIFY,
};

// Returns 1 if the input nIn of the serialized transaction correctly spends scriptPubKey.
__attribute__((visibility("default"))) int bitcoinconsensus_verify_script(
    const uint8_t* scriptPubKey, unsigned int scriptPubKeyLen, const uint8_t* txTo, unsigned int txToLen,
    unsigned int nIn, unsigned int flags, bitcoinconsensus_error* err);

__attribute__((visibility("default"))) int bitcoinconsensus_verify_script_with_amount(
    const uint8_t* scriptPubKey, unsigned int scriptPubKeyLen, int64_t amount, const uint8_t* txTo,
    unsigned int txToLen, unsigned int nIn, unsigned int flags, bitcoinconsensus_error* err);

__attribute__((visibility("default"))) unsigned int bitcoinconsensus_version();

#ifdef __cplusplus
}
#endif
