// Proof of work: difficulty schedule and checks.
// Parity: reference src/pow.{h,cpp}
//   GetNextWorkRequired     pow.cpp:71   genesis -> powLimit(false); regtest no-retarget;
//                                        pre-fork legacy 2016-block retarget; premine window ->
//                                        powLimit; averaging window -> powLimitStart; else DAA
//   CalculateNextWorkRequired pow.cpp:105 (legacy)
//   CheckProofOfWork        pow.cpp:141  (range check against PowLimit(postfork))
//   GetNextCashPlusWorkRequired pow.cpp:252 (144-block work-weighted DAA, median-of-3)
//   CheckEquihashSolution   pow.cpp:298
#pragma once
#include "consensus/chain.h"
#include "consensus/params.h"

#include <vector>

namespace bcp {

uint32_t GetNextWorkRequired(const CBlockIndex* pindexPrev, const CBlockHeader* pblock,
                             const Consensus::Params& params);
uint32_t CalculateNextWorkRequired(const CBlockIndex* pindexPrev, int64_t nFirstBlockTime,
                                   const Consensus::Params& params);
uint32_t GetNextCashPlusWorkRequired(const CBlockIndex* pindexPrev, const CBlockHeader* pblock,
                                     const Consensus::Params& params);
bool CheckProofOfWork(const uint256& hash, uint32_t nBits, bool postfork, const Consensus::Params& params);

// CPU consensus check of one header's Equihash solution.
bool CheckEquihashSolution(const CBlockHeader* pblock, const CChainParams& params);
// Batched check (GPU when available, CPU otherwise); result[i] for headers[i].
std::vector<bool> CheckEquihashSolutions(const std::vector<const CBlockHeader*>& headers, const CChainParams& params,
                                         bool allow_gpu = true);

} // namespace bcp
