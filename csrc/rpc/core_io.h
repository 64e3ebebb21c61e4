// Hex/JSON codecs for transactions, blocks and scripts.
// Parity: reference src/core_read.cpp (DecodeHexTx, DecodeHexBlk with the legacy
// header flag, ParseHashStr, ParseSighashString) and src/core_write.cpp
// (FormatScript, ScriptToAsmStr, EncodeHexTx, ScriptPubKeyToUniv, TxToUniv).
#pragma once
#include "consensus/chain.h"
#include "primitives/block.h"
#include "util/univalue.h"

namespace bcp {

class CChainParams;

bool DecodeHexTx(CMutableTransaction& tx, const std::string& strHexTx);
bool DecodeHexBlk(CBlock& block, const std::string& strHexBlk, bool fLegacyFormat = false);
bool DecodeHexBlockHeader(CBlockHeader& header, const std::string& hex, bool fLegacyFormat = false);
std::string EncodeHexTx(const CTransaction& tx);
std::string EncodeHexBlock(const CBlock& block, bool fLegacyFormat);
uint256 ParseHashStr(const std::string& str, const std::string& name);
int ParseSighashString(const std::string& s); // "ALL|FORKID" etc.; throws
std::string FormatScript(const CScript& script);
void ScriptPubKeyToUniv(const CScript& scriptPubKey, UniValue& out, bool fIncludeHex, const CChainParams& params);
// fRpcSize: include "size" like the RPC TxToJSON (reference rpc/rawtransaction.cpp:65); the
// core_write.cpp TxToUniv used by bitcoin-tx and REST omits it.
void TxToUniv(const CTransaction& tx, const uint256& hashBlock, UniValue& entry, const CChainParams& params,
              bool fRpcSize = true);
double GetDifficultyFromBits(uint32_t nBits);

} // namespace bcp
