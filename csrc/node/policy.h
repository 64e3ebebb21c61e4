// Relay/mining policy: standardness, dust, fee-rate globals.
// Parity: reference src/policy/policy.{h,cpp} (IsStandard: bare multisig n<=3,
// OP_RETURN size/datacarrier; IsStandardTx: version, size, scriptSig size 1650 and
// push-only, dust, one OP_RETURN; AreInputsStandard: P2SH sigops <= 15;
// GetDustThreshold 3 * fee(size + 148)) and src/primitives/transaction.h IsDust.
#pragma once
#include "node/coins.h"
#include "primitives/amount.h"
#include "script/standard.h"

#include <string>

namespace bcp {

static const uint64_t DEFAULT_MAX_GENERATED_BLOCK_SIZE = 2 * 1000000;
static const uint64_t DEFAULT_BLOCK_PRIORITY_PERCENTAGE = 5;
static const Amount DEFAULT_BLOCK_MIN_TX_FEE = 1000;
static const unsigned int MAX_STANDARD_TX_SIZE = 100000;
static const unsigned int MAX_P2SH_SIGOPS = 15;
static const unsigned int MAX_STANDARD_TX_SIGOPS = 20000 / 5;
static const unsigned int DEFAULT_MAX_MEMPOOL_SIZE = 300; // MB
static const Amount DEFAULT_INCREMENTAL_RELAY_FEE = 1000;
static const unsigned int DEFAULT_BYTES_PER_SIGOP = 20;
static const Amount DUST_RELAY_TX_FEE = 1000;
static const bool DEFAULT_PERMIT_BAREMULTISIG = true;
static const bool DEFAULT_RELAYPRIORITY = true;
static const unsigned int DEFAULT_LIMITFREERELAY = 0;
static const bool DEFAULT_ACCEPT_DATACARRIER = true;

extern CFeeRate incrementalRelayFee;
extern CFeeRate dustRelayFee;
extern CFeeRate minRelayTxFee;
extern unsigned int nBytesPerSigOp;
extern bool fIsBareMultisigStd;
extern bool fRequireStandard;

bool IsStandard(const CScript& scriptPubKey, txnouttype& whichType);
bool IsStandardTx(const CTransaction& tx, std::string& reason);
bool AreInputsStandard(const CTransaction& tx, const CCoinsViewCache& mapInputs);
Amount GetDustThreshold(const CTxOut& txout, const CFeeRate& dustRelayFee);
inline bool IsDust(const CTxOut& txout, const CFeeRate& fee) { return txout.nValue < GetDustThreshold(txout, fee); }

// Coin-age priority (reference src/coins.cpp GetPriority / txmempool AllowFree).
double GetPriority(const CTransaction& tx, const CCoinsViewCache& view, int nHeight, Amount& inChainInputValue);
inline bool AllowFree(double dPriority) { return dPriority > double(COIN) * 144 / 250; }

} // namespace bcp
