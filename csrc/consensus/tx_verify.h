// Context-free and UTXO-contextual transaction checks.
// Parity: reference src/validation.cpp
//   IsFinalTx :233, CalculateSequenceLocks :261, EvaluateSequenceLocks :331,
//   SequenceLocks :341, GetSigOpCountWithoutP2SH :435, GetP2SHSigOpCount :446,
//   GetTransactionSigOpCount :462, CheckTransactionCommon :476, CheckCoinbase :532,
//   CheckRegularTransaction :551, Consensus::CheckTxInputs :1368;
//   src/consensus/consensus.h (size/sigop limits, COINBASE_MATURITY, LOCKTIME_* flags).
#pragma once
#include "consensus/chain.h"
#include "consensus/validation_state.h"
#include "primitives/transaction.h"

#include <utility>
#include <vector>

namespace bcp {

static const uint64_t ONE_MEGABYTE = 1000000;
static const uint64_t MAX_TX_SIZE = ONE_MEGABYTE;
static const uint64_t LEGACY_MAX_BLOCK_SIZE = ONE_MEGABYTE;
static const uint64_t DEFAULT_MAX_BLOCK_SIZE = 8 * ONE_MEGABYTE;
static const int64_t MAX_BLOCK_SIGOPS_PER_MB = 20000;
static const uint64_t MAX_TX_SIGOPS_COUNT = 20000;
static const int COINBASE_MATURITY = 100;
enum { LOCKTIME_VERIFY_SEQUENCE = (1 << 0), LOCKTIME_MEDIAN_TIME_PAST = (1 << 1) };
static const unsigned int STANDARD_LOCKTIME_VERIFY_FLAGS = LOCKTIME_VERIFY_SEQUENCE | LOCKTIME_MEDIAN_TIME_PAST;

inline uint64_t GetMaxBlockSigOpsCount(uint64_t blockSize) {
    const uint64_t nMbRoundedUp = 1 + ((blockSize - 1) / ONE_MEGABYTE);
    return nMbRoundedUp * MAX_BLOCK_SIGOPS_PER_MB;
}

class CCoinsViewCache;

bool IsFinalTx(const CTransaction& tx, int nBlockHeight, int64_t nBlockTime);
std::pair<int, int64_t> CalculateSequenceLocks(const CTransaction& tx, int flags, std::vector<int>* prevHeights,
                                               const CBlockIndex& block);
bool EvaluateSequenceLocks(const CBlockIndex& block, std::pair<int, int64_t> lockPair);
bool SequenceLocks(const CTransaction& tx, int flags, std::vector<int>* prevHeights, const CBlockIndex& block);

uint64_t GetSigOpCountWithoutP2SH(const CTransaction& tx);
uint64_t GetP2SHSigOpCount(const CTransaction& tx, const CCoinsViewCache& inputs);
uint64_t GetTransactionSigOpCount(const CTransaction& tx, const CCoinsViewCache& inputs, int flags);

bool CheckCoinbase(const CTransaction& tx, CValidationState& state, bool fCheckDuplicateInputs = true);
bool CheckRegularTransaction(const CTransaction& tx, CValidationState& state, bool fCheckDuplicateInputs = true);

namespace Consensus {
bool CheckTxInputs(const CTransaction& tx, CValidationState& state, const CCoinsViewCache& inputs, int nSpendHeight);
}

} // namespace bcp
