// Consensus parameters and per-network chain parameters.
// Parity: reference src/consensus/params.h:41-91 and src/chainparams.{h,cpp}:95-472
// (main/test/regtest: BCP fork heights, premine window, pow limits, Equihash (N,K),
// magic bytes, ports, genesis assertions, checkpoints, base58/CashAddr prefixes).
#pragma once
#include "primitives/amount.h"
#include "primitives/block.h"
#include "primitives/uint256.h"

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace bcp {
namespace Consensus {

enum DeploymentPos { DEPLOYMENT_TESTDUMMY, DEPLOYMENT_CSV, MAX_VERSION_BITS_DEPLOYMENTS };

struct BIP9Deployment {
    int bit = 0;
    int64_t nStartTime = 0;
    int64_t nTimeout = 0;
};

struct Params {
    uint256 hashGenesisBlock;
    int nSubsidyHalvingInterval = 210000;
    int BIP34Height = 0;
    uint256 BIP34Hash;
    int BIP65Height = 0;
    int BIP66Height = 0;
    int BCPHeight = 0;               // Equihash + new header from this height
    int BCPPremineWindow = 0;        // blocks mined at powLimit right after the fork
    int antiReplayOpReturnSunsetHeight = 0;
    std::vector<unsigned char> antiReplayOpReturnCommitment;
    uint32_t nRuleChangeActivationThreshold = 0;
    uint32_t nMinerConfirmationWindow = 0;
    BIP9Deployment vDeployments[MAX_VERSION_BITS_DEPLOYMENTS];
    uint256 powLimit, powLimitLegacy, powLimitStart;
    bool fPowAllowMinDifficultyBlocks = false;
    bool fPowNoRetargeting = false;
    int64_t nPowTargetSpacing = 600;
    int64_t nPowTargetTimespanLegacy = 14 * 24 * 60 * 60;
    int64_t nPowAveragingWindow = 30;
    uint256 nMinimumChainWork;
    uint256 defaultAssumeValid;
    int64_t DifficultyAdjustmentInterval() const { return nPowTargetTimespanLegacy / nPowTargetSpacing; }
    const uint256& PowLimit(bool postfork) const { return postfork ? powLimit : powLimitLegacy; }
};

} // namespace Consensus

struct CDNSSeedData {
    std::string name, host;
    bool supportsServiceBitsFiltering;
};

// A fixed seed node: 16-byte IPv6-form address (IPv4 v4-mapped, onion in the OnionCat prefix)
// and port (reference chainparamsseeds.h / SeedSpec6).
struct SeedSpec6 {
    uint8_t addr[16];
    uint16_t port;
};

struct CCheckpointData {
    std::map<int, uint256> mapCheckpoints;
};

struct ChainTxData {
    int64_t nTime;
    int64_t nTxCount;
    double dTxRate;
};

class CChainParams {
public:
    enum Base58Type { PUBKEY_ADDRESS, SCRIPT_ADDRESS, SECRET_KEY, EXT_PUBLIC_KEY, EXT_SECRET_KEY, MAX_BASE58_TYPES };

    const Consensus::Params& GetConsensus() const { return consensus; }
    Consensus::Params& MutableConsensus() { return consensus; }
    const unsigned char* NetMagic() const { return netMagic; }
    const unsigned char* DiskMagic() const { return diskMagic; }
    int GetDefaultPort() const { return nDefaultPort; }
    int GetRPCPort() const { return nRPCPort; }
    const CBlock& GenesisBlock() const { return genesis; }
    bool MiningRequiresPeers() const { return fMiningRequiresPeers; }
    bool DefaultConsistencyChecks() const { return fDefaultConsistencyChecks; }
    bool RequireStandard() const { return fRequireStandard; }
    uint64_t PruneAfterHeight() const { return nPruneAfterHeight; }
    unsigned int EquihashN() const { return nEquihashN; }
    unsigned int EquihashK() const { return nEquihashK; }
    bool MineBlocksOnDemand() const { return fMineBlocksOnDemand; }
    const std::string& NetworkIDString() const { return strNetworkID; }
    const std::string& DataDirSuffix() const { return strDataDir; }
    const std::vector<CDNSSeedData>& DNSSeeds() const { return vSeeds; }
    const std::vector<SeedSpec6>& FixedSeeds() const { return vFixedSeeds; }
    const std::vector<unsigned char>& Base58Prefix(Base58Type t) const { return base58Prefixes[t]; }
    const std::string& CashAddrPrefix() const { return cashaddrPrefix; }
    const CCheckpointData& Checkpoints() const { return checkpointData; }
    const ChainTxData& TxData() const { return chainTxData; }
    void UpdateVersionBitsParameters(Consensus::DeploymentPos d, int64_t nStart, int64_t nTimeout) {
        consensus.vDeployments[d].nStartTime = nStart;
        consensus.vDeployments[d].nTimeout = nTimeout;
    }

protected:
    CChainParams() {}
    Consensus::Params consensus;
    unsigned char netMagic[4] = {0, 0, 0, 0};
    unsigned char diskMagic[4] = {0, 0, 0, 0};
    int nDefaultPort = 0;
    int nRPCPort = 0;
    uint64_t nPruneAfterHeight = 0;
    unsigned int nEquihashN = 0, nEquihashK = 0;
    std::vector<CDNSSeedData> vSeeds;
    std::vector<SeedSpec6> vFixedSeeds;
    std::vector<unsigned char> base58Prefixes[MAX_BASE58_TYPES];
    std::string cashaddrPrefix;
    std::string strNetworkID, strDataDir;
    CBlock genesis;
    bool fMiningRequiresPeers = true;
    bool fDefaultConsistencyChecks = false;
    bool fRequireStandard = true;
    bool fMineBlocksOnDemand = false;
    CCheckpointData checkpointData;
    ChainTxData chainTxData{0, 0, 0};
    friend std::unique_ptr<CChainParams> CreateChainParams(const std::string& chain);
};

std::unique_ptr<CChainParams> CreateChainParams(const std::string& chain);
const CChainParams& Params();
CChainParams& Params(const std::string& chain);
void SelectParams(const std::string& chain);
bool ChainParamsSelected();

// Subsidy schedule (reference src/validation.cpp:1169 GetBlockSubsidy).
Amount GetBlockSubsidy(int nHeight, const Consensus::Params& params);

} // namespace bcp
