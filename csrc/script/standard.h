// Standard output templates and destinations.
// Parity: reference src/script/standard.{h,cpp} (txnouttype, Solver :43-150,
// ExtractDestination(s) :152-210, GetScriptFor* :212-261, MAX_OP_RETURN_RELAY = 83).
#pragma once
#include "keys/key.h"
#include "script/script.h"

#include <vector>

namespace bcp {

static const unsigned int MAX_OP_RETURN_RELAY = 83;
extern bool fAcceptDatacarrier;
extern unsigned nMaxDatacarrierBytes;

enum txnouttype { TX_NONSTANDARD, TX_PUBKEY, TX_PUBKEYHASH, TX_SCRIPTHASH, TX_MULTISIG, TX_NULL_DATA };

const char* GetTxnOutputType(txnouttype t);
bool Solver(const CScript& scriptPubKey, txnouttype& typeRet, std::vector<std::vector<unsigned char>>& solutions);
bool ExtractDestination(const CScript& scriptPubKey, CTxDestination& addressRet);
bool ExtractDestinations(const CScript& scriptPubKey, txnouttype& typeRet, std::vector<CTxDestination>& addressRet,
                         int& nRequiredRet);
CScript GetScriptForDestination(const CTxDestination& dest);
CScript GetScriptForRawPubKey(const CPubKey& pubkey);
CScript GetScriptForMultisig(int nRequired, const std::vector<CPubKey>& keys);

} // namespace bcp
