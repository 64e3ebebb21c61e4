#include "consensus/pow.h"
#include "consensus/equihash.h"
#include "crypto/common.h"
#include "kernels/gpu_api.h"
#include "node/gpuverify.h"
#include "util/util.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>

namespace bcp {

static uint32_t BitcoinGetNextWorkRequired(const CBlockIndex* pindexLast, const CBlockHeader* pblock,
                                           const Consensus::Params& params) {
    const uint32_t nProofOfWorkLimit = UintToArith256(params.PowLimit(false)).GetCompact();
    if (pindexLast == nullptr) return nProofOfWorkLimit;
    const int64_t interval = params.DifficultyAdjustmentInterval();
    if ((pindexLast->nHeight + 1) % interval != 0) {
        if (params.fPowAllowMinDifficultyBlocks) {
            // testnet: a block more than 2x the spacing late may use the minimum difficulty
            if (pblock->GetBlockTime() > pindexLast->GetBlockTime() + params.nPowTargetSpacing * 2)
                return nProofOfWorkLimit;
            const CBlockIndex* p = pindexLast;
            while (p->pprev && p->nHeight % interval != 0 && p->nBits == nProofOfWorkLimit) p = p->pprev;
            return p->nBits;
        }
        return pindexLast->nBits;
    }
    const int nHeightFirst = pindexLast->nHeight - (int)(interval - 1);
    const CBlockIndex* pindexFirst = pindexLast->GetAncestor(nHeightFirst);
    return CalculateNextWorkRequired(pindexLast, pindexFirst->GetBlockTime(), params);
}

uint32_t GetNextWorkRequired(const CBlockIndex* pindexPrev, const CBlockHeader* pblock,
                             const Consensus::Params& params) {
    if (pindexPrev == nullptr) return UintToArith256(params.PowLimit(false)).GetCompact();
    if (params.fPowNoRetargeting) return pindexPrev->nBits;
    const int nHeight = pindexPrev->nHeight + 1;
    const bool postfork = nHeight >= params.BCPHeight;
    if (!postfork) return BitcoinGetNextWorkRequired(pindexPrev, pblock, params);
    if (nHeight < params.BCPHeight + params.BCPPremineWindow)
        return UintToArith256(params.PowLimit(true)).GetCompact();
    if (nHeight < params.BCPHeight + params.BCPPremineWindow + params.nPowAveragingWindow)
        return UintToArith256(params.powLimitStart).GetCompact();
    return GetNextCashPlusWorkRequired(pindexPrev, pblock, params);
}

uint32_t CalculateNextWorkRequired(const CBlockIndex* pindexPrev, int64_t nFirstBlockTime,
                                   const Consensus::Params& params) {
    if (params.fPowNoRetargeting) return pindexPrev->nBits;
    int64_t span = pindexPrev->GetBlockTime() - nFirstBlockTime;
    span = std::max(span, params.nPowTargetTimespanLegacy / 4);
    span = std::min(span, params.nPowTargetTimespanLegacy * 4);
    const arith_uint256 bnPowLimit = UintToArith256(params.PowLimit(false));
    arith_uint256 bnNew;
    bnNew.SetCompact(pindexPrev->nBits);
    bnNew *= (uint32_t)span;
    bnNew /= arith_uint256((uint64_t)params.nPowTargetTimespanLegacy);
    if (bnNew > bnPowLimit) bnNew = bnPowLimit;
    return bnNew.GetCompact();
}

bool CheckProofOfWork(const uint256& hash, uint32_t nBits, bool postfork, const Consensus::Params& params) {
    bool fNegative, fOverflow;
    arith_uint256 bnTarget;
    bnTarget.SetCompact(nBits, &fNegative, &fOverflow);
    if (fNegative || bnTarget == 0 || fOverflow || bnTarget > UintToArith256(params.PowLimit(postfork))) return false;
    return UintToArith256(hash) <= bnTarget;
}

// Work done between two blocks scaled to the target spacing, bounded to [72, 288] spacings.
static arith_uint256 ComputeTarget(const CBlockIndex* pindexFirst, const CBlockIndex* pindexLast,
                                   const Consensus::Params& params) {
    arith_uint256 work = pindexLast->nChainWork - pindexFirst->nChainWork;
    work *= (uint32_t)params.nPowTargetSpacing;
    int64_t span = (int64_t)pindexLast->nTime - (int64_t)pindexFirst->nTime;
    if (span > 288 * params.nPowTargetSpacing) span = 288 * params.nPowTargetSpacing;
    else if (span < 72 * params.nPowTargetSpacing) span = 72 * params.nPowTargetSpacing;
    work /= arith_uint256((uint64_t)span);
    // T = 2^256 / W - 1 computed as (2^256 - W) / W
    return (-work) / work;
}

// Median (by timestamp) of the block and its two predecessors.
static const CBlockIndex* GetSuitableBlock(const CBlockIndex* pindex) {
    const CBlockIndex* b[3] = {pindex->pprev->pprev, pindex->pprev, pindex};
    if (b[0]->nTime > b[2]->nTime) std::swap(b[0], b[2]);
    if (b[0]->nTime > b[1]->nTime) std::swap(b[0], b[1]);
    if (b[1]->nTime > b[2]->nTime) std::swap(b[1], b[2]);
    return b[1];
}

uint32_t GetNextCashPlusWorkRequired(const CBlockIndex* pindexPrev, const CBlockHeader* pblock,
                                     const Consensus::Params& params) {
    const bool postfork = pindexPrev->nHeight >= params.BCPHeight;
    if (params.fPowAllowMinDifficultyBlocks &&
        pblock->GetBlockTime() > pindexPrev->GetBlockTime() + 2 * params.nPowTargetSpacing)
        return UintToArith256(params.PowLimit(postfork)).GetCompact();
    const uint32_t nHeight = pindexPrev->nHeight;
    const CBlockIndex* pindexLast = GetSuitableBlock(pindexPrev);
    const CBlockIndex* pindexFirst = GetSuitableBlock(pindexPrev->GetAncestor(nHeight - 144));
    const arith_uint256 nextTarget = ComputeTarget(pindexFirst, pindexLast, params);
    const arith_uint256 powLimit = UintToArith256(params.PowLimit(postfork));
    if (nextTarget > powLimit) return powLimit.GetCompact();
    return nextTarget.GetCompact();
}

// CEquihashInput || nNonce (140 bytes) without a temporary vector.
static void WriteEquihashInput(const CBlockHeader& h, uint8_t* out) {
    auto le32 = [&](uint32_t v) {
        WriteLE32(out, v);
        out += 4;
    };
    le32((uint32_t)h.nVersion);
    memcpy(out, h.hashPrevBlock.begin(), 32);
    memcpy(out + 32, h.hashMerkleRoot.begin(), 32);
    out += 64;
    le32(h.nHeight);
    for (int i = 0; i < 7; ++i) le32(h.nReserved[i]);
    le32(h.nTime);
    le32(h.nBits);
    memcpy(out, h.nNonce.begin(), 32);
}

static CBlake2b EquihashStateFor(const CBlockHeader* pblock, const EquihashParams& ep) {
    CBlake2b st = EhInitialiseState(ep);
    std::vector<unsigned char> in = pblock->EquihashInput();
    st.Write(in.data(), in.size());
    st.Write(pblock->nNonce.begin(), 32);
    return st;
}

bool CheckEquihashSolution(const CBlockHeader* pblock, const CChainParams& params) {
    const EquihashParams ep(params.EquihashN(), params.EquihashK());
    return EhIsValidSolution(ep, EquihashStateFor(pblock, ep), pblock->nSolution);
}

std::vector<bool> CheckEquihashSolutions(const std::vector<const CBlockHeader*>& headers, const CChainParams& params,
                                         bool allow_gpu) {
    const EquihashParams ep(params.EquihashN(), params.EquihashK());
    std::vector<bool> out(headers.size(), false);
    if (headers.empty()) return out;
    static std::atomic<int> gpuFailures{0};
    if (allow_gpu && headers.size() >= 4 && gpuFailures.load() < 3 && (GpuFaultInjection() || gpu::GpuAvailable())) {
        // A device failure must not leave headers neither accepted nor rejected: log it and
        // verify the same batch on the CPU. Three consecutive failures turn the GPU path off.
        try {
            if (GpuFaultInjection()) throw std::runtime_error("injected GPU Equihash-verify fault");
            // raw header bytes straight into each lane's pinned staging (its own fill workers); the
            // device builds the BLAKE2b base states (no host hashing), sharded across the
            // validation GPUs (node/gpuverify.h)
            const size_t solBytes = gpu::EquihashSolutionBytes(ep.N, ep.K);
            auto fill = [&](size_t lo, size_t hi, uint8_t* in, uint8_t* sols, uint8_t* lenok, WorkerPool& workers) {
                workers.ParallelFor(
                    hi - lo,
                    [&](size_t k) {
                        const CBlockHeader& h = *headers[lo + k];
                        WriteEquihashInput(h, in + k * 140);
                        const bool ok = h.nSolution.size() == solBytes;
                        lenok[k] = ok;
                        if (ok) memcpy(sols + k * solBytes, h.nSolution.data(), solBytes);
                        else memset(sols + k * solBytes, 0, solBytes);
                    },
                    32);
            };
            std::vector<uint8_t> r = GpuVerifyService::Instance().EquihashHeaders(ep.N, ep.K, headers.size(), fill);
            for (size_t i = 0; i < r.size(); ++i) out[i] = r[i] != 0;
            gpuFailures = 0;
            return out;
        } catch (const std::exception& e) {
            const int f = ++gpuFailures;
            LogPrintf("GPU Equihash verification failed (%s); verifying %zu headers on the CPU%s\n", e.what(),
                      headers.size(), f >= 3 ? " (GPU path now disabled)" : "");
        }
    }
    for (size_t i = 0; i < headers.size(); ++i) out[i] = EhIsValidSolution(ep, EquihashStateFor(headers[i], ep), headers[i]->nSolution);
    return out;
}

} // namespace bcp
