// Chainstate engine: block index, header/block acceptance, connect/disconnect with
// undo, best-chain activation and reorgs, flushing, mempool acceptance.
//
// Parity map (reference src/validation.cpp):
//   CheckBlockHeader :3202 (Equihash at header nHeight >= BCPHeight, PoW vs PowLimit(postfork))
//   CheckBlock :3222, ContextualCheckBlockHeader :3362 (bad-diffbits, bad-height, time rules,
//   bad-version), ContextualCheckTransaction :3413 (anti-replay commitment until sunset),
//   ContextualCheckBlock :3474 (BIP34 coinbase height), AcceptBlockHeader :3519,
//   AcceptBlock :3615, ProcessNewBlock :3736, ProcessNewBlockHeaders :3590,
//   TestBlockValidity :3774, GetBlockScriptFlags :1803 (FORKID always, STRICTENC|LOW_S|NULLFAIL
//   post-fork, ALLOW_NON_FORKID pre-fork), ConnectBlock :1868 (script failures ignored before
//   the fork, :2124), DisconnectBlock/ApplyBlockUndo :1634-1714, FlushStateToDisk :2196,
//   UpdateTip :2348, DisconnectTip :2435, ConnectTip :2525, FindMostWorkChain :2598,
//   ActivateBestChainStep :2678, ActivateBestChain :2793, PreciousBlock :2889,
//   InvalidateBlock :2919, ResetBlockFailureFlags :2967, AddToBlockIndex :3005,
//   ReceivedBlockTransactions :3049, FindBlockPos :3104, LoadBlockIndexDB :4033,
//   VerifyDB :4167, RewindBlockIndex :4324, InitBlockIndex :4412, LoadExternalBlockFile :4461,
//   CheckBlockIndex :4618, AcceptToMemoryPoolWorker :666, LoadMempool/DumpMempool :4948-5070,
//   GuessVerificationProgress :5073, IsInitialBlockDownload :1180.
//
// MI355X design: ConnectBlock evaluates all input scripts on the CPU worker pool with a
// DeferringSignatureChecker, then verifies the collected ECDSA checks in one batch on the
// GPU (csrc/kernels/secp256k1.hip) when the batch is large enough. Headers arriving in
// bulk (ProcessNewBlockHeaders) have their Equihash solutions verified as one GPU batch.
#pragma once
#include "consensus/chain.h"
#include "consensus/params.h"
#include "consensus/tx_verify.h"
#include "consensus/validation_state.h"
#include "consensus/versionbits.h"
#include "node/coins.h"
#include "node/txdb.h"
#include "util/checkqueue.h"
#include "util/util.h"

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>

namespace bcp {

class CTxMemPool;
struct LockPoints;

static const int64_t DEFAULT_MAX_TIP_AGE = 24 * 60 * 60;
static const unsigned int MIN_BLOCKS_TO_KEEP = 288;
static const int DEFAULT_CHECKBLOCKS = 6;
static const unsigned int DEFAULT_CHECKLEVEL = 3;
static const uint64_t MIN_DISK_SPACE_FOR_BLOCK_FILES = 550 * 1024 * 1024;
static const int MAX_SCRIPTCHECK_THREADS = 64;
static const unsigned int DATABASE_WRITE_INTERVAL = 60 * 60;
static const unsigned int DATABASE_FLUSH_INTERVAL = 24 * 60 * 60;
static const uint64_t MIN_TRANSACTION_SIZE = 10; // smallest serialisable tx with one in/out: guards vtx count
static const unsigned int DEFAULT_ANCESTOR_LIMIT = 25;
static const unsigned int DEFAULT_ANCESTOR_SIZE_LIMIT = 101;
static const unsigned int DEFAULT_DESCENDANT_LIMIT = 25;
static const unsigned int DEFAULT_DESCENDANT_SIZE_LIMIT = 101;
static const unsigned int DEFAULT_MEMPOOL_EXPIRY = 336;
static const Amount DEFAULT_MIN_RELAY_TX_FEE = 1000; // per kB
static const Amount DEFAULT_TRANSACTION_MAXFEE = COIN / 10;

enum FlushStateMode { FLUSH_STATE_NONE, FLUSH_STATE_IF_NEEDED, FLUSH_STATE_PERIODIC, FLUSH_STATE_ALWAYS };
enum DisconnectResult { DISCONNECT_OK, DISCONNECT_UNCLEAN, DISCONNECT_FAILED };

// Reverts a connected block's coin changes from its undo record: its outputs are spent, the
// coins its inputs spent come back, and the view's best block becomes the block's parent
// (reference src/validation.cpp ApplyBlockUndo, the part of DisconnectBlock after the undo read).
DisconnectResult ApplyBlockUndo(const CBlockUndo& blockUndo, const CBlock& block, const CBlockIndex* pindex,
                                CCoinsViewCache& view);
// Spends tx's inputs (recording the spent coins in txundo) and adds its outputs at nHeight
// (reference UpdateCoins); the inputs must exist in the view.
void UpdateCoins(const CTransaction& tx, CCoinsViewCache& view, CTxUndo& txundo, int nHeight);
void UpdateCoins(const CTransaction& tx, CCoinsViewCache& view, int nHeight);

struct ChainstateOptions {
    std::string datadir;            // <datadir> (net specific); blocks/ chainstate/ blocks/index/
    bool memoryOnly = false;        // in-memory databases (tests)
    bool wipe = false;              // -reindex / fresh start
    size_t coinsCacheBytes = 450u << 20;
    bool txindex = false;
    int scriptThreads = 0;          // <= 0: auto (cores)
    bool useGpu = true;             // batch ECDSA + header Equihash verification on the GPU
    bool checkBlockIndex = false;   // -checkblockindex (expensive consistency checks)
    bool checkpoints = true;
    uint64_t maxBlockSize = DEFAULT_MAX_BLOCK_SIZE;
    uint64_t pruneTarget = 0;       // bytes; 0 = no pruning
    uint256 assumeValid;
    int64_t maxTipAge = DEFAULT_MAX_TIP_AGE;
    // the UTXO pass of a block with at least this many transactions runs in parallel (0: never)
    size_t parallelUtxoMinTx = 64;
    // that pass updates the coins tip in place (undone from the undo records if a later check
    // fails) instead of a per-block view merged into the tip afterwards (-connectinplace)
    bool connectInPlace = true;
    // with the tip updated in place and the signatures on the GPU, the next block's read-only
    // pass runs meanwhile on the idle script threads (-connectlookahead)
    bool connectLookahead = true;
    // -blockcachemb: blocks accepted but not yet connected stay in memory up to this many
    // serialized bytes (oldest evicted first), so the connect that follows (IBD, blocks arriving
    // out of order) skips the disk read, the deserialisation and the repeat CheckBlock; 0: off
    size_t recentBlockBytes = 512u << 20;
};

// Mempool acceptance outcome.
struct MempoolAcceptResult {
    bool accepted = false;
    bool missingInputs = false;
    Amount fee = 0;
};

// A block's undo record serialised for disk (the bytes of SerializeToBytes(undo, SER_DISK)),
// transaction chunks in parallel on `pool` when given.
std::vector<unsigned char> SerializeBlockUndo(const CBlockUndo& undo, WorkerPool* pool);
// GetSerializeSize(block, version) from the transactions' cached sizes.
uint64_t BlockSerializeSize(const CBlock& block, int version);
// -maxscriptcachesize (MiB): resize the script-execution cache; returns its capacity.
size_t InitScriptExecutionCache(int64_t mib);
// UI alert + -alertnotify command.
void AlertNotify(const std::string& strMessage);

class Chainstate {
public:
    Chainstate(const CChainParams& params, const ChainstateOptions& opts);
    ~Chainstate();
    Chainstate(const Chainstate&) = delete;

    // ---- lifecycle
    bool LoadBlockIndex(std::string& err);  // block tree + chain tip from disk
    bool InitBlockIndex(std::string& err);  // genesis when empty
    bool ReplayBlocks(std::string& err);    // recover from an interrupted UTXO flush
    bool RewindBlockIndex();                // drop blocks validated without the current rules
    bool VerifyDB(int nCheckLevel, int nCheckDepth);
    bool LoadExternalBlockFile(FILE* fileIn, CDiskBlockPos* dbp = nullptr);
    bool Reindex();                         // re-import all blk*.dat files
    void Shutdown();                        // final flush

    // ---- block processing
    bool ProcessNewBlock(const std::shared_ptr<const CBlock>& block, bool fForceProcessing, bool* fNewBlock,
                         CValidationState* stateOut = nullptr);
    bool ProcessNewBlockHeaders(const std::vector<CBlockHeader>& headers, CValidationState& state,
                                const CBlockIndex** ppindex = nullptr);
    bool ActivateBestChain(CValidationState& state, std::shared_ptr<const CBlock> pblock = nullptr);
    bool TestBlockValidity(CValidationState& state, const CBlock& block, CBlockIndex* pindexPrev, bool fCheckPOW,
                           bool fCheckMerkleRoot);
    bool InvalidateBlock(CValidationState& state, CBlockIndex* pindex);
    bool ResetBlockFailureFlags(CBlockIndex* pindex);
    bool PreciousBlock(CValidationState& state, CBlockIndex* pindex);
    bool FlushStateToDisk(CValidationState& state, FlushStateMode mode, int nManualPruneHeight = 0);
    void FlushStateToDisk();
    void PruneBlockFilesManual(int nManualPruneHeight);

    // context-free / contextual checks (also used by the miner and RPC)
    bool CheckBlockHeader(const CBlockHeader& block, CValidationState& state, bool fCheckPOW = true) const;
    bool CheckBlock(const CBlock& block, CValidationState& state, bool fCheckPOW = true,
                    bool fCheckMerkleRoot = true) const;
    bool ContextualCheckBlockHeader(const CBlockHeader& block, CValidationState& state, const CBlockIndex* pindexPrev,
                                    int64_t nAdjustedTime) const;
    bool ContextualCheckTransaction(const CTransaction& tx, CValidationState& state, int nHeight,
                                    int64_t nLockTimeCutoff) const;
    bool ContextualCheckTransactionForCurrentBlock(const CTransaction& tx, CValidationState& state,
                                                   int flags = -1) const EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ContextualCheckBlock(const CBlock& block, CValidationState& state, const CBlockIndex* pindexPrev) const;
    uint32_t GetBlockScriptFlags(const CBlockIndex* pindex) const;
    bool IsBCPEnabled(int nHeight) const { return nHeight >= params.GetConsensus().BCPHeight; }
    bool IsBCPEnabled(const CBlockIndex* pindexPrev) const {
        return pindexPrev != nullptr && IsBCPEnabled(pindexPrev->nHeight);
    }

    // ---- mempool
    void SetMempool(CTxMemPool* pool) { mempool = pool; }
    CTxMemPool* Mempool() const { return mempool; }
    bool AcceptToMemoryPool(CValidationState& state, const CTransactionRef& tx, bool fLimitFree,
                            bool* pfMissingInputs, bool fOverrideMempoolLimit = false, Amount nAbsurdFee = 0,
                            int64_t nAcceptTime = 0, Amount* feeOut = nullptr);
    bool CheckSequenceLocks(const CTransaction& tx, int flags, LockPoints* lp = nullptr,
                            bool useExistingLockPoints = false) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool TestLockPointValidity(const LockPoints* lp) const EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool LoadMempool(const std::string& path);
    bool DumpMempool(const std::string& path);
    void LimitMempoolSize(size_t limit, unsigned long age);

    // ---- queries
    CCriticalSection& cs() const RETURN_CAPABILITY(cs_main) { return cs_main; }
    const CChainParams& Params() const { return params; }
    CChain& ActiveChain() EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return chainActive; }
    const CChain& ActiveChain() const EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return chainActive; }
    CBlockIndex* Tip() const EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return chainActive.Tip(); }
    int Height() const EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return chainActive.Height(); }
    // Tip height for code that does not hold cs_main (takes it; not while holding a mempool lock,
    // cs_main is always taken first)
    int HeightNow() const {
        std::lock_guard<CCriticalSection> l(cs_main);
        return chainActive.Height();
    }
    CBlockIndex* TipNow() const {
        std::lock_guard<CCriticalSection> l(cs_main);
        return chainActive.Tip();
    }
    CBlockIndex* BestHeader() const EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return pindexBestHeader; }
    CBlockIndex* LookupBlockIndex(const uint256& hash) const;
    const BlockMap& BlockIndex() const EXCLUSIVE_LOCKS_REQUIRED(cs_main) { return mapBlockIndex; }
    CCoinsViewCache& CoinsTip() { return *pcoinsTip; }
    CCoinsViewDB& CoinsDB() { return *pcoinsdbview; }
    CBlockTreeDB& BlockTree() { return *pblocktree; }
    bool IsInitialBlockDownload() const;
    bool ReadBlock(CBlock& block, const CBlockIndex* pindex, bool checkPow = true) const;
    bool GetTransaction(const uint256& txid, CTransactionRef& txOut, uint256& hashBlock, bool fAllowSlow);
    CBlockIndex* FindForkInGlobalIndex(const CBlockLocator& locator) const;
    std::vector<const CBlockIndex*> GetChainTips() const;
    double GuessVerificationProgress(const CBlockIndex* pindex) const;
    ThresholdState DeploymentState(const CBlockIndex* pindexPrev, Consensus::DeploymentPos pos);
    int32_t ComputeBlockVersion(const CBlockIndex* pindexPrev);
    VersionBitsCache& VersionBits() { return versionbitscache; }
    uint64_t MaxBlockSize() const { return opts.maxBlockSize; }
    // Sizes up to the legacy 1 MB limit are refused and leave the setting unchanged (reference
    // GlobalConfig::SetMaxBlockSize, src/config.cpp).
    bool SetMaxBlockSize(uint64_t n) {
        if (n <= LEGACY_MAX_BLOCK_SIZE) return false;
        opts.maxBlockSize = n;
        return true;
    }
    bool TxIndexEnabled() const { return opts.txindex; }
    bool PruneMode() const { return opts.pruneTarget > 0; }
    bool HavePruned() const { return fHavePruned; }
    uint64_t CalculateCurrentUsage() const;
    WorkerPool& Pool() { return *pool; }
    bool UseGpu() const { return opts.useGpu; }
    void SetUseGpu(bool v) { opts.useGpu = v; }
    void SetParallelUtxoMinTx(size_t n) { opts.parallelUtxoMinTx = n; }
    std::string Warnings() const; // bcp::GetWarnings("statusbar")
    // block-change notification for RPC long-poll / waitfornewblock
    void WaitForBlockChange(int64_t timeoutMillis, const uint256& from);
    std::condition_variable_any& BlockChangeCV() { return cvBlockChange; }
    int64_t LastBlockConnectMicros() const { return nLastConnectMicros; }
    // Cumulative wall time (microseconds) of ConnectBlockPrepare's phases, for -debug=bench and
    // the connect benchmarks: CheckBlock, the parallel read-only pass (BIP30, input prefetch,
    // per-tx precompute), the serial UTXO pass, the wait for
    // the script jobs after it, gathering the deferred checks, and the synchronous batch verify.
    // PH_BLOCKS counts connected blocks, PH_FASTUTXO those whose UTXO pass took the parallel path;
    // PH_FU_* split that parallel pass (setup, checks, undo + jobs, view updates; inside PH_UTXO)
    // PH_ABC_* split ActivateBestChain (reference validation.cpp:2678-2873) around ConnectTip:
    // FindMostWorkChain, the steps (PH_ABC_TIP: the ConnectTip calls inside them), the
    // BlockConnected signals, the hand-off of the connected blocks to the reaper, the tip
    // notifications, CheckBlockIndex and the periodic flush; PH_ACCEPT is AcceptBlock inside
    // ProcessNewBlock (CheckBlock, contextual checks, the write to disk).
    enum ConnectPhase {
        PH_CHECK, PH_PRECOMPUTE, PH_UTXO, PH_SCRIPTS, PH_COLLECT, PH_BATCH, PH_BLOCKS, PH_FASTUTXO,
        PH_FU_SETUP, PH_FU_CHECKS, PH_FU_UNDO, PH_FU_APPLY,
        PH_ABC_FIND, PH_ABC_STEP, PH_ABC_TIP, PH_ABC_SIGNALS, PH_ABC_REAP, PH_ABC_NOTIFY, PH_ABC_CHECKINDEX,
        PH_ABC_FLUSH, PH_ACCEPT,
        // inside ConnectTip (and the pipelined commit): block read from disk, ConnectBlock
        // (prepare + finish), view flush into the coins tip, FlushStateToDisk, mempool + tip update
        PH_TIP_READ, PH_TIP_CONNECT, PH_TIP_FLUSH, PH_TIP_WRITE, PH_TIP_POST,
        PH_UNDO, // inside ConnectBlockFinish: the block's undo data serialised and written
        // the connect lookahead: time the connecting thread waited for it after block N's
        // verdict, and the number of blocks whose connect adopted it (a count, not micros)
        PH_LA_WAIT, PH_LA_USED,
        PH_COUNT
    };
    int64_t ConnectPhaseMicros(ConnectPhase ph) const { return phaseMicros[ph].load(std::memory_order_relaxed); }
    // connects that found their block in the recent-block cache / had to read it from disk
    uint64_t RecentBlockHits() const { return recentHits.load(std::memory_order_relaxed); }
    uint64_t RecentBlockMisses() const { return recentMisses.load(std::memory_order_relaxed); }

private:
    struct WorkComparator {
        bool operator()(const CBlockIndex* a, const CBlockIndex* b) const;
    };
    struct ConnectTrace {
        std::vector<std::pair<CBlockIndex*, std::shared_ptr<const CBlock>>> blocksConnected;
    };

    CBlockIndex* InsertBlockIndex(const uint256& hash) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    CBlockIndex* AddToBlockIndex(const CBlockHeader& block) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool AcceptBlockHeader(const CBlockHeader& block, CValidationState& state, CBlockIndex** ppindex,
                           bool skipPow = false) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool AcceptBlock(const std::shared_ptr<const CBlock>& pblock, CValidationState& state, CBlockIndex** ppindex,
                     bool fRequested, const CDiskBlockPos* dbp, bool* fNewBlock) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ReceivedBlockTransactions(const CBlock& block, CValidationState& state, CBlockIndex* pindexNew,
                                   const CDiskBlockPos& pos) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool FindBlockPos(CValidationState& state, CDiskBlockPos& pos, unsigned nAddSize, unsigned nHeight,
                      uint64_t nTime, bool fKnown = false) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool FindUndoPos(CValidationState& state, int nFile, CDiskBlockPos& pos, unsigned nAddSize) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void FlushBlockFile(bool fFinalize = false);
    struct PendingConnect; // a block between its UTXO pass and its signature verdict
    bool ConnectBlockPrepare(const CBlock& block, CValidationState& state, CBlockIndex* pindex, CCoinsViewCache& view,
                             bool fJustCheck, PendingConnect& p) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ConnectBlockFinish(PendingConnect& p, CValidationState& state, bool fJustCheck)
        EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ConnectBlock(const CBlock& block, CValidationState& state, CBlockIndex* pindex, CCoinsViewCache& view,
                      bool fJustCheck = false, CCoinsViewCache* directTip = nullptr) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    DisconnectResult DisconnectBlock(const CBlock& block, const CBlockIndex* pindex, CCoinsViewCache& view) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool DisconnectTip(CValidationState& state, bool fBare = false) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ConnectTip(CValidationState& state, CBlockIndex* pindexNew, const std::shared_ptr<const CBlock>& pblock,
                    ConnectTrace& trace) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    CBlockIndex* FindMostWorkChain() EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void PruneBlockIndexCandidates() EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool ActivateBestChainStep(CValidationState& state, CBlockIndex* pindexMostWork,
                               const std::shared_ptr<const CBlock>& pblock, bool& fInvalidFound, ConnectTrace& trace) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void UpdateTip(CBlockIndex* pindexNew) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void InvalidChainFound(CBlockIndex* pindexNew) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void InvalidBlockFound(CBlockIndex* pindex, const CValidationState& state) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void CheckBlockIndex(); // takes cs_main itself
    bool LoadBlockIndexDB(std::string& err) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool LoadChainTip() EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void NotifyHeaderTip();
    bool CheckIndexAgainstCheckpoint(const CBlockIndex* pindexPrev, CValidationState& state) const;
    void FindFilesToPrune(std::set<int>& setFilesToPrune, uint64_t nPruneAfterHeight) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void FindFilesToPruneManual(std::set<int>& setFilesToPrune, int nManualPruneHeight) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void PruneOneBlockFile(int fileNumber) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void UnlinkPrunedFiles(const std::set<int>& setFilesToPrune);
    bool CheckInputs(const CTransaction& tx, CValidationState& state, const CCoinsViewCache& inputs,
                     bool fScriptChecks, uint32_t flags, bool cacheStore, const PrecomputedTransactionData& txdata)
        EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool AcceptToMemoryPoolWorker(CValidationState& state, const CTransactionRef& ptx, bool fLimitFree,
                                  bool* pfMissingInputs, int64_t nAcceptTime, bool fOverrideMempoolLimit,
                                  Amount nAbsurdFee, std::vector<COutPoint>& coins_to_uncache, Amount* feeOut) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void UpdateMempoolForReorg(const std::vector<CTransactionRef>& disconnected, bool fAddToMempool) EXCLUSIVE_LOCKS_REQUIRED(cs_main);

    const CChainParams& params;
    ChainstateOptions opts;
    mutable CCriticalSection cs_main{"cs_main"};
    std::condition_variable_any cvBlockChange;

    BlockMap mapBlockIndex GUARDED_BY(cs_main);
    std::vector<std::unique_ptr<CBlockIndex>> blockIndexStorage;
    std::vector<std::unique_ptr<uint256>> hashStorage;
    CChain chainActive GUARDED_BY(cs_main);
    CBlockIndex* pindexBestHeader GUARDED_BY(cs_main) = nullptr;
    CBlockIndex* pindexBestInvalid = nullptr;
    void CheckForkWarningConditions() EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void CheckForkWarningConditionsOnNewFork(CBlockIndex* pindexNewForkTip) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void RemoveForReorgAtTip() EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    CBlockIndex* pindexBestForkTip = nullptr;
    CBlockIndex* pindexBestForkBase = nullptr;
    std::set<CBlockIndex*, WorkComparator> setBlockIndexCandidates GUARDED_BY(cs_main);
    std::multimap<CBlockIndex*, CBlockIndex*> mapBlocksUnlinked GUARDED_BY(cs_main);
    std::set<CBlockIndex*> setDirtyBlockIndex GUARDED_BY(cs_main);
    std::set<int> setDirtyFileInfo GUARDED_BY(cs_main);
    std::vector<CBlockFileInfo> vinfoBlockFile;
    int nLastBlockFile = 0;
    int32_t nBlockSequenceId = 1;
    int32_t nBlockReverseSequenceId = -1;
    arith_uint256 nLastPreciousChainwork = 0;
    bool fHavePruned = false;
    bool fCheckForPruning = false;
    bool fReindex = false;
    mutable std::atomic<bool> latchToFalse{false};
    int64_t nLastWrite = 0, nLastFlush = 0, nLastSetChain = 0;
    std::atomic<int64_t> nLastConnectMicros{0};
    std::atomic<int64_t> phaseMicros[PH_COUNT] = {};
    // accepted, not yet connected blocks (ChainstateOptions::recentBlockBytes), by block hash
    void CacheRecentBlock(const uint256& hash, const std::shared_ptr<const CBlock>& pblock, size_t bytes)
        EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    std::shared_ptr<const CBlock> TakeRecentBlock(const uint256& hash) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    std::shared_ptr<const CBlock> PeekRecentBlock(const uint256& hash) const EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    // Connect lookahead: while block N's signatures are on the GPU, the script threads run block
    // N+1's read-only pass (its input coins fetched from the tip, which already holds N's
    // in-place update; sighash midstates, sizes, sigop counts). N+1's connect adopts the result
    // when nothing changed in between; a failed N, a disconnect or any other block drops it.
    struct BlockPrefetch;
    struct Lookahead;
    std::unique_ptr<Lookahead> lookahead;
    CBlockIndex* pindexConnectNext = nullptr; // the block ActivateBestChainStep connects after this one
    void StartLookahead(const CBlockIndex* pindex) EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    void JoinLookahead();
    bool ScriptChecksFor(const CBlockIndex* pindex) const EXCLUSIVE_LOCKS_REQUIRED(cs_main);
    bool EnforceBIP30For(const CBlockIndex* pindex) const;
    std::map<uint256, std::pair<std::shared_ptr<const CBlock>, size_t>> recentBlocks GUARDED_BY(cs_main);
    std::deque<uint256> recentOrder GUARDED_BY(cs_main);
    size_t recentBytes GUARDED_BY(cs_main) = 0;
    std::atomic<uint64_t> recentHits{0}, recentMisses{0};

    std::unique_ptr<CBlockTreeDB> pblocktree;
    std::unique_ptr<CCoinsViewDB> pcoinsdbview;
    std::unique_ptr<CCoinsViewCache> pcoinsTip;
    std::unique_ptr<WorkerPool> pool;
    std::unique_ptr<CheckQueue> scriptQueue; // ConnectBlock script checks (reference CCheckQueue)
    VersionBitsCache versionbitscache;
    ThresholdConditionCache warningcache[VERSIONBITS_NUM_BITS]; // unknown-versionbit tracking (cs_main)
    bool fUnknownRulesWarned = false;
    CTxMemPool* mempool = nullptr;
};

// Process-wide node chainstate (RPC, P2P and the wallet reach it through here).
Chainstate* GetChainstate();
void SetChainstate(Chainstate* cs);

std::string FormatStateMessage(const CValidationState& state);

} // namespace bcp
