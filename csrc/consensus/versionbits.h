// BIP9 version-bits deployment state machine.
// Parity: reference src/versionbits.{h,cpp} (ThresholdState, AbstractThresholdConditionChecker
// GetStateFor/GetStateSinceHeightFor with per-period cache, VersionBitsState/Mask) and
// ComputeBlockVersion src/validation.cpp:1750.
#pragma once
#include "consensus/chain.h"
#include "consensus/params.h"

#include <map>
#include <mutex>

namespace bcp {

static const int32_t VERSIONBITS_LAST_OLD_BLOCK_VERSION = 4;
static const int32_t VERSIONBITS_TOP_BITS = 0x20000000UL;
static const int32_t VERSIONBITS_TOP_MASK = 0xE0000000UL;
static const int32_t VERSIONBITS_NUM_BITS = 29;

enum ThresholdState { THRESHOLD_DEFINED, THRESHOLD_STARTED, THRESHOLD_LOCKED_IN, THRESHOLD_ACTIVE, THRESHOLD_FAILED };
const char* ThresholdStateName(ThresholdState s);

typedef std::map<const CBlockIndex*, ThresholdState> ThresholdConditionCache;

struct BIP9Stats {
    int period = 0, threshold = 0, elapsed = 0, count = 0;
    bool possible = false;
};

class AbstractThresholdConditionChecker {
public:
    virtual ~AbstractThresholdConditionChecker() {}
    virtual bool Condition(const CBlockIndex* pindex, const Consensus::Params& params) const = 0;
    virtual int64_t BeginTime(const Consensus::Params& params) const = 0;
    virtual int64_t EndTime(const Consensus::Params& params) const = 0;
    virtual int Period(const Consensus::Params& params) const = 0;
    virtual int Threshold(const Consensus::Params& params) const = 0;
    ThresholdState GetStateFor(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                               ThresholdConditionCache& cache) const;
    int GetStateSinceHeightFor(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                               ThresholdConditionCache& cache) const;
    BIP9Stats GetStateStatisticsFor(const CBlockIndex* pindex, const Consensus::Params& params) const;
};

struct VersionBitsCache {
    ThresholdConditionCache caches[Consensus::MAX_VERSION_BITS_DEPLOYMENTS];
    std::mutex cs;
    void Clear();
};

ThresholdState VersionBitsState(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos, VersionBitsCache& cache);
int VersionBitsStateSinceHeight(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos, VersionBitsCache& cache);
BIP9Stats VersionBitsStatistics(const CBlockIndex* pindexPrev, const Consensus::Params& params,
                                Consensus::DeploymentPos pos);
uint32_t VersionBitsMask(const Consensus::Params& params, Consensus::DeploymentPos pos);
int32_t ComputeBlockVersion(const CBlockIndex* pindexPrev, const Consensus::Params& params, VersionBitsCache& cache);

struct VBDeploymentInfo {
    const char* name;
    bool gbt_force;
};
extern const VBDeploymentInfo VersionBitsDeploymentInfo[Consensus::MAX_VERSION_BITS_DEPLOYMENTS];

} // namespace bcp
