#include "consensus/chain.h"
#include "consensus/params.h"
#include "util/strencodings.h"

namespace bcp {

CBlockHeader CBlockIndex::GetBlockHeader() const {
    CBlockHeader block;
    block.nVersion = nVersion;
    if (pprev) block.hashPrevBlock = pprev->GetBlockHash();
    block.hashMerkleRoot = hashMerkleRoot;
    block.nHeight = nHeight;
    memcpy(block.nReserved, nReserved, sizeof(block.nReserved));
    block.nTime = nTime;
    block.nBits = nBits;
    block.nNonce = nNonce;
    block.nSolution = nSolution;
    return block;
}

CBlockHeader CDiskBlockIndex::GetHeader() const {
    CBlockHeader block;
    block.nVersion = nVersion;
    block.hashPrevBlock = hashPrev;
    block.hashMerkleRoot = hashMerkleRoot;
    block.nHeight = nHeight;
    memcpy(block.nReserved, nReserved, sizeof(block.nReserved));
    block.nTime = nTime;
    block.nBits = nBits;
    block.nNonce = nNonce;
    block.nSolution = nSolution;
    return block;
}

int64_t CBlockIndex::GetMedianTimePast() const {
    int64_t pmedian[nMedianTimeSpan];
    int n = 0;
    const CBlockIndex* p = this;
    for (int i = 0; i < nMedianTimeSpan && p; i++, p = p->pprev) pmedian[n++] = p->GetBlockTime();
    std::sort(pmedian, pmedian + n);
    return pmedian[n / 2];
}

std::string CBlockIndex::ToString() const {
    return strprintf("CBlockIndex(pprev=%p, nHeight=%d, merkle=%s, hashBlock=%s)", (void*)pprev, nHeight,
                     hashMerkleRoot.ToString().c_str(), phashBlock ? GetBlockHash().ToString().c_str() : "null");
}

static inline int InvertLowestOne(int n) { return n & (n - 1); }
static inline int GetSkipHeight(int height) {
    if (height < 2) return 0;
    return (height & 1) ? InvertLowestOne(InvertLowestOne(height - 1)) + 1 : InvertLowestOne(height);
}

CBlockIndex* CBlockIndex::GetAncestor(int height) {
    if (height > nHeight || height < 0) return nullptr;
    CBlockIndex* walk = this;
    int hw = nHeight;
    while (hw > height) {
        int hs = GetSkipHeight(hw);
        int hsp = GetSkipHeight(hw - 1);
        if (walk->pskip != nullptr && (hs == height || (hs > height && !(hsp < hs - 2 && hsp >= height)))) {
            walk = walk->pskip;
            hw = hs;
        } else {
            walk = walk->pprev;
            hw--;
        }
    }
    return walk;
}

const CBlockIndex* CBlockIndex::GetAncestor(int height) const { return const_cast<CBlockIndex*>(this)->GetAncestor(height); }

void CBlockIndex::BuildSkip() {
    if (pprev) pskip = pprev->GetAncestor(GetSkipHeight(nHeight));
}

arith_uint256 GetBlockProof(const CBlockIndex& block) {
    arith_uint256 bnTarget;
    bool fNegative, fOverflow;
    bnTarget.SetCompact(block.nBits, &fNegative, &fOverflow);
    if (fNegative || fOverflow || bnTarget == 0) return 0;
    return (~bnTarget / (bnTarget + 1)) + 1;
}

int64_t GetBlockProofEquivalentTime(const CBlockIndex& to, const CBlockIndex& from, const CBlockIndex& tip,
                                    const Consensus::Params& params) {
    arith_uint256 r;
    int sign = 1;
    if (to.nChainWork > from.nChainWork) {
        r = to.nChainWork - from.nChainWork;
    } else {
        r = from.nChainWork - to.nChainWork;
        sign = -1;
    }
    r = r * arith_uint256(params.nPowTargetSpacing) / GetBlockProof(tip);
    if (r.bits() > 63) return sign * std::numeric_limits<int64_t>::max();
    return sign * (int64_t)r.GetLow64();
}

const CBlockIndex* LastCommonAncestor(const CBlockIndex* pa, const CBlockIndex* pb) {
    if (pa->nHeight > pb->nHeight) pa = pa->GetAncestor(pb->nHeight);
    else if (pb->nHeight > pa->nHeight) pb = pb->GetAncestor(pa->nHeight);
    while (pa != pb && pa && pb) {
        pa = pa->pprev;
        pb = pb->pprev;
    }
    return pa;
}

void CChain::SetTip(CBlockIndex* pindex) {
    if (pindex == nullptr) {
        vChain.clear();
        return;
    }
    vChain.resize(pindex->nHeight + 1);
    while (pindex && vChain[pindex->nHeight] != pindex) {
        vChain[pindex->nHeight] = pindex;
        pindex = pindex->pprev;
    }
}

CBlockLocator CChain::GetLocator(const CBlockIndex* pindex) const {
    int nStep = 1;
    std::vector<uint256> vHave;
    vHave.reserve(32);
    if (!pindex) pindex = Tip();
    while (pindex) {
        vHave.push_back(pindex->GetBlockHash());
        if (pindex->nHeight == 0) break;
        int h = std::max(pindex->nHeight - nStep, 0);
        if (Contains(pindex)) pindex = (*this)[h];
        else pindex = pindex->GetAncestor(h);
        if (vHave.size() > 10) nStep *= 2;
    }
    return CBlockLocator(vHave);
}

const CBlockIndex* CChain::FindFork(const CBlockIndex* pindex) const {
    if (pindex == nullptr) return nullptr;
    if (pindex->nHeight > Height()) pindex = pindex->GetAncestor(Height());
    while (pindex && !Contains(pindex)) pindex = pindex->pprev;
    return pindex;
}

CBlockIndex* CChain::FindEarliestAtLeast(int64_t nTime) const {
    auto lower = std::lower_bound(vChain.begin(), vChain.end(), nTime,
                                  [](CBlockIndex* b, const int64_t& t) { return b->GetBlockTimeMax() < t; });
    return lower == vChain.end() ? nullptr : *lower;
}

} // namespace bcp
