#include "consensus/versionbits.h"

#include <vector>

namespace bcp {

const VBDeploymentInfo VersionBitsDeploymentInfo[Consensus::MAX_VERSION_BITS_DEPLOYMENTS] = {
    {"testdummy", true},
    {"csv", true},
};

const char* ThresholdStateName(ThresholdState s) {
    switch (s) {
    case THRESHOLD_DEFINED: return "defined";
    case THRESHOLD_STARTED: return "started";
    case THRESHOLD_LOCKED_IN: return "locked_in";
    case THRESHOLD_ACTIVE: return "active";
    case THRESHOLD_FAILED: return "failed";
    }
    return "";
}

ThresholdState AbstractThresholdConditionChecker::GetStateFor(const CBlockIndex* pindexPrev,
                                                              const Consensus::Params& params,
                                                              ThresholdConditionCache& cache) const {
    const int nPeriod = Period(params);
    const int nThreshold = Threshold(params);
    const int64_t nTimeStart = BeginTime(params);
    const int64_t nTimeTimeout = EndTime(params);

    // states are constant within a period: evaluate at the last block of the previous period
    if (pindexPrev != nullptr) pindexPrev = pindexPrev->GetAncestor(pindexPrev->nHeight - ((pindexPrev->nHeight + 1) % nPeriod));

    std::vector<const CBlockIndex*> toCompute;
    while (cache.count(pindexPrev) == 0) {
        if (pindexPrev == nullptr) {
            cache[pindexPrev] = THRESHOLD_DEFINED;
            break;
        }
        if (pindexPrev->GetMedianTimePast() < nTimeStart) {
            // optimisation: nothing can have happened before the start time
            cache[pindexPrev] = THRESHOLD_DEFINED;
            break;
        }
        toCompute.push_back(pindexPrev);
        pindexPrev = pindexPrev->GetAncestor(pindexPrev->nHeight - nPeriod);
    }

    ThresholdState state = cache[pindexPrev];
    while (!toCompute.empty()) {
        ThresholdState stateNext = state;
        pindexPrev = toCompute.back();
        toCompute.pop_back();
        switch (state) {
        case THRESHOLD_DEFINED:
            if (pindexPrev->GetMedianTimePast() >= nTimeTimeout) stateNext = THRESHOLD_FAILED;
            else if (pindexPrev->GetMedianTimePast() >= nTimeStart) stateNext = THRESHOLD_STARTED;
            break;
        case THRESHOLD_STARTED: {
            if (pindexPrev->GetMedianTimePast() >= nTimeTimeout) {
                stateNext = THRESHOLD_FAILED;
                break;
            }
            const CBlockIndex* pindexCount = pindexPrev;
            int count = 0;
            for (int i = 0; i < nPeriod; i++) {
                if (Condition(pindexCount, params)) count++;
                pindexCount = pindexCount->pprev;
            }
            if (count >= nThreshold) stateNext = THRESHOLD_LOCKED_IN;
            break;
        }
        case THRESHOLD_LOCKED_IN:
            stateNext = THRESHOLD_ACTIVE;
            break;
        case THRESHOLD_FAILED:
        case THRESHOLD_ACTIVE:
            break;
        }
        cache[pindexPrev] = state = stateNext;
    }
    return state;
}

int AbstractThresholdConditionChecker::GetStateSinceHeightFor(const CBlockIndex* pindexPrev,
                                                              const Consensus::Params& params,
                                                              ThresholdConditionCache& cache) const {
    const ThresholdState initialState = GetStateFor(pindexPrev, params, cache);
    if (initialState == THRESHOLD_DEFINED) return 0;
    const int nPeriod = Period(params);
    pindexPrev = pindexPrev->GetAncestor(pindexPrev->nHeight - ((pindexPrev->nHeight + 1) % nPeriod));
    const CBlockIndex* previousPeriodParent = pindexPrev->GetAncestor(pindexPrev->nHeight - nPeriod);
    while (previousPeriodParent != nullptr && GetStateFor(previousPeriodParent, params, cache) == initialState) {
        pindexPrev = previousPeriodParent;
        previousPeriodParent = pindexPrev->GetAncestor(pindexPrev->nHeight - nPeriod);
    }
    return pindexPrev->nHeight + 1;
}

BIP9Stats AbstractThresholdConditionChecker::GetStateStatisticsFor(const CBlockIndex* pindex,
                                                                   const Consensus::Params& params) const {
    BIP9Stats stats;
    stats.period = Period(params);
    stats.threshold = Threshold(params);
    if (pindex == nullptr) return stats;
    // first block of pindex's period; in the very first period there is no previous-period end block
    const int periodStart = pindex->nHeight - ((pindex->nHeight + 1) % stats.period) + 1;
    stats.elapsed = pindex->nHeight - periodStart + 1;
    int count = 0;
    for (const CBlockIndex* cur = pindex; cur != nullptr && cur->nHeight >= periodStart; cur = cur->pprev)
        if (Condition(cur, params)) count++;
    stats.count = count;
    stats.possible = (stats.period - stats.threshold) >= (stats.elapsed - count);
    return stats;
}

namespace {
class VersionBitsConditionChecker : public AbstractThresholdConditionChecker {
public:
    explicit VersionBitsConditionChecker(Consensus::DeploymentPos id) : id(id) {}
    int64_t BeginTime(const Consensus::Params& p) const override { return p.vDeployments[id].nStartTime; }
    int64_t EndTime(const Consensus::Params& p) const override { return p.vDeployments[id].nTimeout; }
    int Period(const Consensus::Params& p) const override { return (int)p.nMinerConfirmationWindow; }
    int Threshold(const Consensus::Params& p) const override { return (int)p.nRuleChangeActivationThreshold; }
    bool Condition(const CBlockIndex* pindex, const Consensus::Params& p) const override {
        return ((pindex->nVersion & VERSIONBITS_TOP_MASK) == VERSIONBITS_TOP_BITS) && (pindex->nVersion & Mask(p)) != 0;
    }
    uint32_t Mask(const Consensus::Params& p) const { return ((uint32_t)1) << p.vDeployments[id].bit; }

private:
    const Consensus::DeploymentPos id;
};
} // namespace

void VersionBitsCache::Clear() {
    std::lock_guard<std::mutex> l(cs);
    for (auto& c : caches) c.clear();
}

ThresholdState VersionBitsState(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos, VersionBitsCache& cache) {
    std::lock_guard<std::mutex> l(cache.cs);
    return VersionBitsConditionChecker(pos).GetStateFor(pindexPrev, params, cache.caches[pos]);
}
int VersionBitsStateSinceHeight(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos, VersionBitsCache& cache) {
    std::lock_guard<std::mutex> l(cache.cs);
    return VersionBitsConditionChecker(pos).GetStateSinceHeightFor(pindexPrev, params, cache.caches[pos]);
}
BIP9Stats VersionBitsStatistics(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos) {
    return VersionBitsConditionChecker(pos).GetStateStatisticsFor(pindexPrev, params);
}
uint32_t VersionBitsMask(const Consensus::Params& params, Consensus::DeploymentPos pos) {
    return VersionBitsConditionChecker(pos).Mask(params);
}

int32_t ComputeBlockVersion(const CBlockIndex* pindexPrev, const Consensus::Params& params, VersionBitsCache& cache) {
    int32_t nVersion = VERSIONBITS_TOP_BITS;
    for (int i = 0; i < (int)Consensus::MAX_VERSION_BITS_DEPLOYMENTS; i++) {
        const ThresholdState st = VersionBitsState(pindexPrev, params, (Consensus::DeploymentPos)i, cache);
        if (st == THRESHOLD_LOCKED_IN || st == THRESHOLD_STARTED) nVersion |= VersionBitsMask(params, (Consensus::DeploymentPos)i);
    }
    return nVersion;
}

} // namespace bcp
