// Per-network parameters (values from reference src/chainparams.cpp:95-432; the code is new).
#include "consensus/chainparamsseeds.h"
#include "consensus/merkle.h"
#include "consensus/params.h"
#include "util/strencodings.h"

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace bcp {

static std::vector<unsigned char> AntiReplayCommitment() {
    static const char* s = "Bitcoin: A Peer-to-Peer Electronic Cash System";
    return std::vector<unsigned char>(s, s + strlen(s));
}

static CBlock MakeGenesis(uint32_t nTime, uint32_t nNonce, uint32_t nBits, int32_t nVersion, Amount reward) {
    const char* ts = "The Times 03/Jan/2009 Chancellor on brink of second bailout for banks";
    CMutableTransaction tx;
    tx.nVersion = 1;
    tx.vin.resize(1);
    tx.vout.resize(1);
    tx.vin[0].scriptSig = CScript() << 486604799 << CScriptNum(4)
                                    << std::vector<unsigned char>((const unsigned char*)ts, (const unsigned char*)ts + strlen(ts));
    tx.vout[0].nValue = reward;
    tx.vout[0].scriptPubKey = CScript() << ParseHex("04678afdb0fe5548271967f1a67130b7105cd6a828e03909a67962e0ea1f61deb649f6"
                                                    "bc3f4cef38c4f35504e51ec112de5c384df7ba0b8d578a4c702b6bf11d5f")
                                        << OP_CHECKSIG;
    CBlock g;
    g.nTime = nTime;
    g.nBits = nBits;
    g.nNonce = ArithToUint256(arith_uint256(nNonce));
    g.nVersion = nVersion;
    g.vtx.push_back(MakeTransactionRef(std::move(tx)));
    g.hashPrevBlock.SetNull();
    g.nHeight = 0;
    g.hashMerkleRoot = BlockMerkleRoot(g);
    return g;
}

class CMainParams : public CChainParams {
public:
    CMainParams() {
        strNetworkID = "main";
        strDataDir = "";
        consensus.nSubsidyHalvingInterval = 210000;
        consensus.BIP34Height = 227931;
        consensus.BIP34Hash = uint256S("000000000000024b89b42a942fe0d9fea3bb44ab7bd1b19115dd6a759c0808b8");
        consensus.BIP65Height = 388381;
        consensus.BIP66Height = 363725;
        consensus.antiReplayOpReturnSunsetHeight = 530000;
        consensus.antiReplayOpReturnCommitment = AntiReplayCommitment();
        consensus.BCPHeight = 509696;
        consensus.BCPPremineWindow = 16000;
        consensus.powLimit = uint256S("7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitStart = uint256S("00000fffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitLegacy = uint256S("00000000ffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.nPowAveragingWindow = 30;
        consensus.nPowTargetTimespanLegacy = 14 * 24 * 60 * 60;
        consensus.nPowTargetSpacing = 10 * 60;
        consensus.fPowAllowMinDifficultyBlocks = false;
        consensus.fPowNoRetargeting = false;
        consensus.nRuleChangeActivationThreshold = 1916;
        consensus.nMinerConfirmationWindow = 2016;
        consensus.vDeployments[Consensus::DEPLOYMENT_TESTDUMMY] = {28, 1199145601, 1230767999};
        consensus.vDeployments[Consensus::DEPLOYMENT_CSV] = {0, 1462060800, 1493596800};
        consensus.nMinimumChainWork = uint256S("0000000000000000000000000000000000000000011c44bff1ea6d8b048a90c2");
        consensus.defaultAssumeValid = uint256S("00000000000000000009fd0c45ae65ff7ac277f05521e6bc19ba08c4f78d0922");
        const unsigned char nm[4] = {0x44, 0x6d, 0x47, 0xe1}, dm[4] = {0xf9, 0xbe, 0xb4, 0xd9};
        memcpy(netMagic, nm, 4);
        memcpy(diskMagic, dm, 4);
        nDefaultPort = 8337;
        nRPCPort = 8332;
        nPruneAfterHeight = 100000;
        nEquihashN = 200;
        nEquihashK = 9;
        genesis = MakeGenesis(1231006505, 2083236893, 0x1d00ffff, 1, 50 * COIN);
        consensus.hashGenesisBlock = genesis.GetHash(consensus);
        if (consensus.hashGenesisBlock != uint256S("000000000019d6689c085ae165831e934ff763ae46a2a6c172b3f1b60a8ce26f") ||
            genesis.hashMerkleRoot != uint256S("4a5e1e4baab89f3a32518a88c31bc87f618f76673e2cc77ab2127b7afdeda33b"))
            throw std::logic_error("main genesis mismatch");
        vSeeds = {{"bcpfork.org", "seed.bcpfork.org", true},
                  {"bcpseeds.net", "seed.bcpseeds.net", true},
                  {"bitcoincashplus.org", "seed.bitcoincashplus.org", true}};
        vFixedSeeds = FixedSeedsMain();
        base58Prefixes[PUBKEY_ADDRESS] = {28};
        base58Prefixes[SCRIPT_ADDRESS] = {23};
        base58Prefixes[SECRET_KEY] = {128};
        base58Prefixes[EXT_PUBLIC_KEY] = {0x04, 0x88, 0xB2, 0x1E};
        base58Prefixes[EXT_SECRET_KEY] = {0x04, 0x88, 0xAD, 0xE4};
        fDefaultConsistencyChecks = false;
        fRequireStandard = true;
        fMineBlocksOnDemand = false;
        fMiningRequiresPeers = true;
        cashaddrPrefix = "bitcoincashplus";
        checkpointData.mapCheckpoints = {
            {11111, uint256S("0000000069e244f73d78e8fd29ba2fd2ed618bd6fa2ee92559f542fdb26e7c1d")},
            {33333, uint256S("000000002dd5588a74784eaa7ab0507a18ad16a236e7b1ce69f00d7ddfb5d0a6")},
            {74000, uint256S("0000000000573993a3c9e41ce34471c079dcf5f52a0e824a81e7f953b8661a20")},
            {105000, uint256S("00000000000291ce28027faea320c8d2b054b2e0fe44a773f3eefb151d6bdc97")},
            {134444, uint256S("00000000000005b12ffd4cd315cd34ffd4a594f430ac814c91184a0d42d2b0fe")},
            {168000, uint256S("000000000000099e61ea72015e79632f216fe6cb33d7899acb35b75c8303b763")},
            {193000, uint256S("000000000000059f452a5f7340de6682a977387c17010ff6e6c3bd83ca8b1317")},
            {210000, uint256S("000000000000048b95347e83192f69cf0366076336c639f9b7228e9ba171342e")},
            {216116, uint256S("00000000000001b4f4b433e81ee46494af945cf96014816a4e2370f11b23df4e")},
            {225430, uint256S("00000000000001c108384350f74090433e7fcf79a606b8e797f065b130575932")},
            {250000, uint256S("000000000000003887df1f29024b06fc2200b55f8af8f35453d7be294df2d214")},
            {279000, uint256S("0000000000000001ae8c72a0b0c301f67e3afca10e819efa9041e458e9bd7e40")},
            {295000, uint256S("00000000000000004d9b4ef50f0f9d686fd69db2e03af35a100370c64632a983")}};
        chainTxData = ChainTxData{1516903077, 295363220, 3.2};
    }
};

class CTestNetParams : public CChainParams {
public:
    CTestNetParams() {
        strNetworkID = "test";
        strDataDir = "testnet3";
        consensus.nSubsidyHalvingInterval = 210000;
        consensus.BIP34Height = 21111;
        consensus.BIP34Hash = uint256S("0000000023b3a96d3484e5abb3755c413e7d41500f8e2a5c3f0dd01299cd8ef8");
        consensus.BIP65Height = 581885;
        consensus.BIP66Height = 330776;
        consensus.BCPHeight = 1257620;
        consensus.BCPPremineWindow = 4500;
        consensus.antiReplayOpReturnSunsetHeight = 1250000;
        consensus.antiReplayOpReturnCommitment = AntiReplayCommitment();
        consensus.powLimit = uint256S("0007ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitStart = uint256S("0000000fffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitLegacy = uint256S("00000000ffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.nPowAveragingWindow = 30;
        consensus.nPowTargetTimespanLegacy = 14 * 24 * 60 * 60;
        consensus.nPowTargetSpacing = 10 * 60;
        consensus.fPowAllowMinDifficultyBlocks = true;
        consensus.fPowNoRetargeting = false;
        consensus.nRuleChangeActivationThreshold = 1512;
        consensus.nMinerConfirmationWindow = 2016;
        consensus.vDeployments[Consensus::DEPLOYMENT_TESTDUMMY] = {28, 1199145601, 1230767999};
        consensus.vDeployments[Consensus::DEPLOYMENT_CSV] = {0, 1456790400, 1493596800};
        consensus.nMinimumChainWork = uint256S("000000000000000000000000000000000000000000000033b230c5ee441a7e83");
        consensus.defaultAssumeValid = uint256S("0004f733e58bea62d694259065d87d20605ef40ef19c116c8e133d8bcd30f4ee");
        const unsigned char nm[4] = {0x45, 0x6d, 0x47, 0xe1}, dm[4] = {0x0b, 0x11, 0x09, 0x07};
        memcpy(netMagic, nm, 4);
        memcpy(diskMagic, dm, 4);
        nDefaultPort = 18337;
        nRPCPort = 18332;
        nPruneAfterHeight = 1000;
        nEquihashN = 200;
        nEquihashK = 9;
        genesis = MakeGenesis(1296688602, 414098458, 0x1d00ffff, 1, 50 * COIN);
        consensus.hashGenesisBlock = genesis.GetHash(consensus);
        if (consensus.hashGenesisBlock != uint256S("000000000933ea01ad0ee984209779baaec3ced90fa3f408719526f8d77f4943"))
            throw std::logic_error("testnet genesis mismatch");
        vSeeds = {{"bcpfork.org", "test-seed.bcpfork.org", true},
                  {"bcpseeds.net", "test-seed.bcpseeds.net", true},
                  {"bitcoincashplus.org", "test-seed.bitcoincashplus.org", true}};
        vFixedSeeds = FixedSeedsTest();
        base58Prefixes[PUBKEY_ADDRESS] = {111};
        base58Prefixes[SCRIPT_ADDRESS] = {196};
        base58Prefixes[SECRET_KEY] = {239};
        base58Prefixes[EXT_PUBLIC_KEY] = {0x04, 0x35, 0x87, 0xCF};
        base58Prefixes[EXT_SECRET_KEY] = {0x04, 0x35, 0x83, 0x94};
        fDefaultConsistencyChecks = false;
        fRequireStandard = false;
        fMineBlocksOnDemand = false;
        fMiningRequiresPeers = true;
        cashaddrPrefix = "bcptest";
        checkpointData.mapCheckpoints = {{546, uint256S("000000002a936ca763904c3c35fce2f3556c559c0214345d31b1bcebf76acb70")}};
        chainTxData = ChainTxData{1501802953, 14706531, 0.15};
    }
};

class CRegTestParams : public CChainParams {
public:
    CRegTestParams() {
        strNetworkID = "regtest";
        strDataDir = "regtest";
        consensus.nSubsidyHalvingInterval = 150;
        consensus.BIP34Height = 100000000;
        consensus.BIP34Hash = uint256();
        consensus.BIP65Height = 1351;
        consensus.BIP66Height = 1251;
        consensus.BCPHeight = 3000;
        consensus.BCPPremineWindow = 20;
        consensus.antiReplayOpReturnSunsetHeight = 530000;
        consensus.antiReplayOpReturnCommitment = AntiReplayCommitment();
        consensus.powLimit = uint256S("7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitStart = uint256S("7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.powLimitLegacy = uint256S("7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff");
        consensus.nPowAveragingWindow = 30;
        consensus.nPowTargetTimespanLegacy = 14 * 24 * 60 * 60;
        consensus.nPowTargetSpacing = 10 * 60;
        consensus.fPowAllowMinDifficultyBlocks = true;
        consensus.fPowNoRetargeting = true;
        consensus.nRuleChangeActivationThreshold = 108;
        consensus.nMinerConfirmationWindow = 144;
        consensus.vDeployments[Consensus::DEPLOYMENT_TESTDUMMY] = {28, 0, 999999999999LL};
        consensus.vDeployments[Consensus::DEPLOYMENT_CSV] = {0, 0, 999999999999LL};
        consensus.nMinimumChainWork = uint256();
        consensus.defaultAssumeValid = uint256();
        const unsigned char nm[4] = {0x46, 0x6d, 0x47, 0xe1}, dm[4] = {0xda, 0xb5, 0xbf, 0xfa};
        memcpy(netMagic, nm, 4);
        memcpy(diskMagic, dm, 4);
        nDefaultPort = 18444;
        nRPCPort = 18332;
        nPruneAfterHeight = 1000;
        nEquihashN = 48;
        nEquihashK = 5;
        genesis = MakeGenesis(1296688602, 2, 0x207fffff, 1, 50 * COIN);
        consensus.hashGenesisBlock = genesis.GetHash(consensus);
        if (consensus.hashGenesisBlock != uint256S("0f9188f13cb7b2c71f2a335e3a4fc328bf5beb436012afca590b1a11466e2206"))
            throw std::logic_error("regtest genesis mismatch");
        fMiningRequiresPeers = false;
        fDefaultConsistencyChecks = true;
        fRequireStandard = false;
        fMineBlocksOnDemand = true;
        checkpointData.mapCheckpoints = {{0, uint256S("0f9188f13cb7b2c71f2a335e3a4fc328bf5beb436012afca590b1a11466e2206")}};
        chainTxData = ChainTxData{0, 0, 0};
        base58Prefixes[PUBKEY_ADDRESS] = {111};
        base58Prefixes[SCRIPT_ADDRESS] = {196};
        base58Prefixes[SECRET_KEY] = {239};
        base58Prefixes[EXT_PUBLIC_KEY] = {0x04, 0x35, 0x87, 0xCF};
        base58Prefixes[EXT_SECRET_KEY] = {0x04, 0x35, 0x83, 0x94};
        cashaddrPrefix = "bcpreg";
    }
};

std::unique_ptr<CChainParams> CreateChainParams(const std::string& chain) {
    if (chain == "main") return std::unique_ptr<CChainParams>(new CMainParams());
    if (chain == "test") return std::unique_ptr<CChainParams>(new CTestNetParams());
    if (chain == "regtest") return std::unique_ptr<CChainParams>(new CRegTestParams());
    throw std::runtime_error("Unknown chain " + chain);
}

static std::mutex g_params_mu;
static std::map<std::string, std::unique_ptr<CChainParams>> g_params;
static CChainParams* g_current = nullptr;

CChainParams& Params(const std::string& chain) {
    std::lock_guard<std::mutex> lk(g_params_mu);
    auto it = g_params.find(chain);
    if (it == g_params.end()) it = g_params.emplace(chain, CreateChainParams(chain)).first;
    return *it->second;
}

void SelectParams(const std::string& chain) { g_current = &Params(chain); }

bool ChainParamsSelected() { return g_current != nullptr; }

const CChainParams& Params() {
    if (!g_current) SelectParams("main");
    return *g_current;
}

Amount GetBlockSubsidy(int nHeight, const Consensus::Params& params) {
    int halvings = nHeight / params.nSubsidyHalvingInterval;
    if (halvings >= 64) return 0;
    Amount nSubsidy = 50 * COIN;
    nSubsidy >>= halvings;
    return nSubsidy;
}

} // namespace bcp
