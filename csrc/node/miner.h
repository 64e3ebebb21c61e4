// Block template assembly and the built-in (GPU) miner.
// Parity: reference src/miner.{h,cpp}: BlockAssembler::CreateNewBlock :137 (coinbase
// `<height> OP_0`, post-fork random 256-bit nonce with top/bottom 16 bits cleared,
// header nHeight/nReserved, TestBlockValidity), addPriorityTxs, addPackageTxs
// (ancestor-feerate packages), ComputeMaxGeneratedBlockSize, IncrementExtraNonce :655
// (`<height> <extranonce> /EB<n>/`), UpdateTime; src/rpc/mining.cpp generateBlocks :115
// (SHA256d nonce loop pre-fork, Equihash solve + target check post-fork).
//
// MI355X: pre-fork headers are swept on the GPU (Sha256dScanNonces) and post-fork
// nonces are solved in batches by the gfx950 Equihash solver; the CPU solver is the
// fallback (and is used for the tiny regtest (48,5) instances where launch latency
// dominates).
#pragma once
#include "node/validation.h"
#include "primitives/block.h"

#include <atomic>
#include <functional>
#include <memory>

namespace bcp {

class CTxMemPool;
class CTxMemPoolEntry;

struct CBlockTemplate {
    CBlock block;
    std::vector<Amount> vTxFees;
    std::vector<int64_t> vTxSigOpsCount;
};

static const bool DEFAULT_PRINTPRIORITY = false;

class BlockAssembler {
public:
    struct Options {
        uint64_t nMaxGeneratedBlockSize;
        CFeeRate blockMinFeeRate;
        int64_t nBlockPriorityPercentage;
        Options();
    };
    BlockAssembler(Chainstate& chainstate, CTxMemPool* mempool, const Options& opts = Options());
    std::unique_ptr<CBlockTemplate> CreateNewBlock(const CScript& scriptPubKeyIn);
    uint64_t LastBlockTx() const { return nLastBlockTx; }
    uint64_t LastBlockSize() const { return nLastBlockSize; }

private:
    void resetBlock();
    void AddToBlock(const CTxMemPoolEntry& e);
    bool TestTxForBlock(const CTransaction& tx, uint64_t size, int64_t sigops) const;
    void addPriorityTxs();
    void addPackageTxs();

    Chainstate& chainstate;
    CTxMemPool* mempool;
    Options options;
    std::unique_ptr<CBlockTemplate> pblocktemplate;
    CBlock* pblock = nullptr;
    std::set<uint256> inBlock;
    uint64_t nBlockSize = 0, nBlockTx = 0, nBlockSigOps = 0;
    Amount nFees = 0;
    int nHeight = 0;
    int64_t nLockTimeCutoff = 0;
    uint64_t nMaxGeneratedBlockSize = 0;
    bool fPrintPriority = false; // -printpriority
    static uint64_t nLastBlockTx, nLastBlockSize;
};

uint64_t ComputeMaxGeneratedBlockSize(uint64_t excessiveBlockSize);
int64_t UpdateTime(CBlockHeader* pblock, const Consensus::Params& params, const CBlockIndex* pindexPrev);
void IncrementExtraNonce(CBlock* pblock, const CBlockIndex* pindexPrev, unsigned& nExtraNonce, uint64_t maxBlockSize);
std::string GetSubVersionEB(uint64_t maxBlockSize); // "8.0" for 8 MB

// Proof-of-work search. Returns true when `block` carries a valid nonce (+ solution);
// nMaxTries counts nonces (legacy) or Equihash instances (post-fork).
struct MinerStats {
    uint64_t sha_nonces = 0, eh_nonces = 0, eh_solutions = 0, blocks = 0;
    double gpu_ms = 0;
};
bool SolveBlock(CBlock& block, const CChainParams& params, uint64_t& nMaxTries, bool useGpu,
                const std::atomic<bool>* cancel = nullptr);
MinerStats GetMinerStats();

// Multi-GPU Equihash search (the built-in miner's post-fork path). Every selected device runs
// two solvers double-buffered on its own host thread; nonces come from one shared counter, so the
// devices sweep disjoint ranges nonce0+1, nonce0+2, ... (nonce-space data parallelism, SURVEY
// §2.3). `accept` is called concurrently from the device threads for every solution found and
// must be thread-safe; the first accepted one ends the search on all devices.
struct EhSearchResult {
    bool found = false;
    uint256 nonce;                        // nonce of the accepted solution
    std::vector<unsigned char> solution;  // minimal encoding
    uint64_t nonces = 0, solutions = 0;   // instances solved / solutions seen (all devices)
};
EhSearchResult EquihashSearchGpu(unsigned n, unsigned k, const std::vector<unsigned char>& equihashInput,
                                 const uint256& nonce0, uint64_t maxNonces,
                                 const std::function<bool(const uint256&, const std::vector<unsigned char>&)>& accept,
                                 std::vector<int> devices = {}, const std::atomic<bool>* cancel = nullptr);
// -gpudevices: devices used by the miner (empty: every visible device).
void SetMinerGpuDevices(const std::vector<int>& devices);
std::vector<int> GetMinerGpuDevices();

// generate / generatetoaddress core: mines nGenerate blocks on the active chain.
std::vector<uint256> GenerateBlocks(Chainstate& chainstate, CTxMemPool* mempool, const CScript& coinbaseScript,
                                    int nGenerate, uint64_t nMaxTries, bool useGpu, std::string* err = nullptr);

} // namespace bcp
