// Chainstate engine: block/header acceptance, connect/disconnect, activation.
// See validation.h for the parity map.
#include "node/validation.h"
#include "node/ui_interface.h"
#include "node/warnings.h"
#include "consensus/merkle.h"
#include "crypto/common.h"
#include "consensus/pow.h"
#include "node/policy.h"
#include "node/signals.h"
#include "node/sigverify.h"
#include "node/txmempool.h"
#include "script/interpreter.h"
#include "util/strencodings.h"
#include "util/memusage.h"
#include "util/reaper.h"

#include <algorithm>
#include <thread>
#include <deque>
#include <future>
#include <tuple>
#include <unistd.h>
#include <cassert>
#include <cmath>

namespace bcp {

static Chainstate* g_chainstate = nullptr;
Chainstate* GetChainstate() { return g_chainstate; }
void SetChainstate(Chainstate* cs) { g_chainstate = cs; }

std::string FormatStateMessage(const CValidationState& state) {
    return strprintf("%s%s (code %i)", state.GetRejectReason().c_str(),
                     state.GetDebugMessage().empty() ? "" : (", " + state.GetDebugMessage()).c_str(),
                     state.GetRejectCode());
}

// Reference validation.cpp AlertNotify: UI alert + -alertnotify=<cmd> with the
// sanitized message single-quoted in place of %s.
void AlertNotify(const std::string& strMessage) {
    uiInterface.NotifyAlertChanged();
    std::string cmd = gArgs.GetArg("-alertnotify", "");
    if (cmd.empty()) return;
    std::string safe = SanitizeString(strMessage);
    safe = safe.substr(0, 200);
    ReplaceAll(cmd, "%s", "'" + safe + "'");
    RunCommandAsync(cmd);
}

// ------------------------------------------------------------------ block-level caches
// Script execution cache: (txid, flags) validated with all inputs (reference
// src/script/scriptcache.cpp). Filled by mempool acceptance, consumed by ConnectBlock.
namespace {
struct ScriptCache {
    SharedCuckooSet set;
    uint256 nonce;
    ScriptCache() {
        GetRandBytes(nonce.begin(), 32);
        set.setup_bytes((size_t)DEFAULT_MAX_SCRIPT_CACHE_SIZE << 20);
    }
    uint256 Key(const CTransaction& tx, uint32_t flags) {
        uint256 r;
        CSHA256().Write(nonce.begin(), 32).Write(tx.GetHash().begin(), 32).Write((const unsigned char*)&flags, 4).Finalize(r.begin());
        return r;
    }
    bool Has(const uint256& k, bool erase) { return set.contains(k, erase); }
    void Add(const uint256& k) {
        if (!everAdded.load(std::memory_order_relaxed)) everAdded.store(true, std::memory_order_relaxed);
        set.insert(k);
    }
    // false while no key was ever added (only mempool acceptance adds): lookups could only miss
    bool MayHold() const { return everAdded.load(std::memory_order_relaxed); }
    std::atomic<bool> everAdded{false};
};
ScriptCache& GetScriptCache() {
    static ScriptCache c;
    return c;
}
} // namespace

// ConnectBlockPrepare's read-only pass over a block, in chunks of transactions that any thread
// may run: BIP30 (no output of the block may already exist unspent), every input's coin fetched
// through `view` (PeekCoins: through the caches to the database without filling them), and the
// per-transaction work that needs no coins - the BIP143-style sighash midstates, the script-cache
// key, the serialized size and the legacy sigop count.
struct Chainstate::BlockPrefetch {
    static constexpr size_t CHUNK = 48; // one batch of coin lookups down the view stack
    std::shared_ptr<const CBlock> hold; // a lookahead's block, kept alive while its chunks run
    const CBlock* block = nullptr;
    const CCoinsView* view = nullptr;
    bool fEnforceBIP30 = false, fScriptChecks = true, scMayHold = false;
    uint32_t flags = 0;
    size_t ntx = 0, maxJobs = 0, nOutputs = 0;
    std::vector<std::unique_ptr<PrecomputedTransactionData>> txdatas;
    std::vector<uint256> scKeys;
    std::vector<uint32_t> txSizes, legacySigOps;
    std::vector<size_t> firstInput; // tx i's inputs are [firstInput[i], firstInput[i+1])
    std::vector<Coin> prefetched;
    std::unique_ptr<uint8_t[]> prefetchedFound;
    std::atomic<bool> bip30Clash{false};

    void Init(const CBlock& b, const CCoinsView& v, bool bip30, bool scripts, bool scHold, uint32_t fl) {
        block = &b;
        view = &v;
        fEnforceBIP30 = bip30;
        fScriptChecks = scripts;
        scMayHold = scHold;
        flags = fl;
        ntx = b.vtx.size();
        txdatas.resize(ntx);
        scKeys.resize(ntx);
        txSizes.resize(ntx);
        legacySigOps.resize(ntx);
        firstInput.assign(ntx + 1, 0);
        nOutputs = 0;
        for (size_t i = 0; i < ntx; i++) {
            firstInput[i + 1] = firstInput[i] + (i > 0 ? b.vtx[i]->vin.size() : 0);
            nOutputs += b.vtx[i]->vout.size();
        }
        maxJobs = firstInput[ntx];
        prefetched.resize(maxJobs);
        prefetchedFound.reset(new uint8_t[maxJobs + 1]);
    }
    size_t Chunks() const { return (ntx + CHUNK - 1) / CHUNK; }
    // Jobs: 0 is Setup, 1.. are the chunks (ParallelFor / script-queue index)
    size_t Jobs() const { return Chunks() + 1; }
    void Job(size_t k, ScriptCache& sc) {
        if (k == 0) Setup();
        else Chunk(k - 1, sc);
    }

    // The parallel UTXO pass's per-block tables, built beside the chunks: the block-local txid
    // index (open addressing; CheckBlock refused duplicate txids), each transaction's first
    // output, each input's transaction, and the zeroed scratch of the in-block spend tracking.
    size_t tcap = 0, scap = 0;
    std::vector<int32_t> tslot;
    std::vector<size_t> firstOutput, inputTx;
    std::unique_ptr<std::atomic<uint8_t>[]> outSpent;  // an output spent inside the block
    std::unique_ptr<std::atomic<uint32_t>[]> spentSet; // concurrent set of spent outpoints
    void Setup() {
        const CBlock& blk = *block;
        tcap = 16;
        while (tcap < 2 * ntx) tcap <<= 1;
        tslot.assign(tcap, -1);
        for (size_t i = 0; i < ntx; i++) {
            size_t h = ReadLE64(blk.vtx[i]->GetHash().begin()) & (tcap - 1);
            while (tslot[h] >= 0) h = (h + 1) & (tcap - 1);
            tslot[h] = (int32_t)i;
        }
        firstOutput.assign(ntx + 1, 0);
        for (size_t i = 0; i < ntx; i++) firstOutput[i + 1] = firstOutput[i] + blk.vtx[i]->vout.size();
        outSpent.reset(new std::atomic<uint8_t>[nOutputs + 1]);
        for (size_t o = 0; o <= nOutputs; o++) outSpent[o].store(0, std::memory_order_relaxed);
        scap = 16;
        while (scap < 2 * maxJobs) scap <<= 1;
        spentSet.reset(new std::atomic<uint32_t>[scap]);
        for (size_t q = 0; q < scap; q++) spentSet[q].store(0, std::memory_order_relaxed);
        inputTx.resize(maxJobs);
        for (size_t i = 1; i < ntx; i++)
            for (size_t k = firstInput[i]; k < firstInput[i + 1]; k++) inputTx[k] = i;
    }
    void Chunk(size_t chunk, ScriptCache& sc) {
        const CBlock& blk = *block;
        const size_t lo = chunk * CHUNK, hi = std::min(ntx, lo + CHUNK);
        std::vector<COutPoint> keys;
        for (size_t i = lo; i < hi; i++) {
            const CTransaction& tx = *blk.vtx[i];
            if (fEnforceBIP30)
                for (size_t o = 0; o < tx.vout.size(); o++) keys.emplace_back(tx.GetHash(), (uint32_t)o);
            if (i > 0)
                for (const CTxIn& in : tx.vin) keys.push_back(in.prevout);
        }
        std::vector<Coin> got(keys.size());
        std::unique_ptr<uint8_t[]> found(new uint8_t[keys.size() + 1]);
        view->PeekCoins(keys.data(), keys.size(), got.data(), found.get());
        size_t q = 0;
        for (size_t i = lo; i < hi; i++) {
            const CTransaction& tx = *blk.vtx[i];
            if (fEnforceBIP30)
                for (size_t o = 0; o < tx.vout.size(); o++, q++)
                    if (found[q] && !got[q].IsSpent()) bip30Clash = true;
            if (i > 0)
                for (size_t k = firstInput[i]; k < firstInput[i + 1]; k++, q++) {
                    prefetchedFound[k] = found[q];
                    if (found[q]) prefetched[k] = std::move(got[q]);
                }
            txSizes[i] = tx.GetTotalSize();
            legacySigOps[i] = (uint32_t)GetSigOpCountWithoutP2SH(tx);
            if (i > 0 && fScriptChecks) {
                if (scMayHold) scKeys[i] = sc.Key(tx, flags);
                txdatas[i].reset(new PrecomputedTransactionData(tx));
            }
        }
    }
};

struct Chainstate::Lookahead {
    uint256 forHash, afterHash; // block N+1, and the block N whose in-place update it read
    BlockPrefetch pf;
    bool open = false; // its chunks are on the script queue (a session this thread must close)
};
size_t InitScriptExecutionCache(int64_t mib) {
    mib = std::min(std::max<int64_t>(0, mib), MAX_MAX_SCRIPT_CACHE_SIZE);
    const size_t n = GetScriptCache().set.setup_bytes((size_t)mib << 20);
    LogPrintf("Using %zu MiB out of %zu requested for script execution cache, able to store %zu elements\n",
              (n * sizeof(uint256)) >> 20, (size_t)mib, n);
    return n;
}
namespace {

// Block validation checker: script logic on the CPU pool, ECDSA deferred to a batch,
// eager checks served from the signature cache when possible.
class BlockSigChecker : public DeferringSignatureChecker {
public:
    BlockSigChecker(const CTransaction* tx, unsigned nIn, Amount amount, const PrecomputedTransactionData* txdata,
                    std::vector<DeferredSigCheck>* sink, std::vector<DeferredMultisig>* groups)
        : DeferringSignatureChecker(tx, nIn, amount, txdata, sink, groups) {}

protected:
    bool VerifySignature(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                         const uint256& sighash) const override {
        SignatureCache& cache = GetSignatureCache();
        const uint256 e = cache.Entry(sighash, sig, pubkey);
        if (cache.Get(e, true)) return true;
        return TransactionSignatureChecker::VerifySignature(sig, pubkey, sighash);
    }
};

struct ScriptJob {
    const CTransaction* tx;
    unsigned nIn;
    const CScript* scriptPubKey; // the spent coin, kept in the block's undo record
    Amount amount;
    const PrecomputedTransactionData* txdata;
};

} // namespace

// ------------------------------------------------------------------ construction
bool Chainstate::WorkComparator::operator()(const CBlockIndex* pa, const CBlockIndex* pb) const {
    if (pa->nChainWork > pb->nChainWork) return false;
    if (pa->nChainWork < pb->nChainWork) return true;
    if (pa->nSequenceId < pb->nSequenceId) return false;
    if (pa->nSequenceId > pb->nSequenceId) return true;
    if (pa < pb) return false;
    if (pa > pb) return true;
    return false;
}

Chainstate::Chainstate(const CChainParams& p, const ChainstateOptions& o) : params(p), opts(o) {
    const std::string base = opts.datadir.empty() ? std::string(".") : opts.datadir;
    if (!opts.memoryOnly) {
        TryCreateDirectories(base + "/blocks");
        SetBlocksDir(base + "/blocks");
    } else {
        TryCreateDirectories(base + "/blocks");
        SetBlocksDir(base + "/blocks");
    }
    // -dbcache split like the reference (init.cpp:1505-1520): a small block-index store cache, the
    // coins store's memtable + block cache, and the rest for the in-memory UTXO cache
    const size_t total = opts.coinsCacheBytes;
    const size_t blockTreeCache = std::min(total / 8, (size_t)2 << 20);
    const size_t coinDBCache = std::min(total / 2, total / 4 + ((size_t)1 << 23));
    opts.coinsCacheBytes = total - blockTreeCache - coinDBCache;
    pblocktree.reset(new CBlockTreeDB(base + "/blocks/index", opts.memoryOnly, opts.wipe, blockTreeCache));
    pcoinsdbview.reset(new CCoinsViewDB(base + "/chainstate", opts.memoryOnly, opts.wipe, coinDBCache));
    pcoinsTip.reset(new CCoinsViewCache(pcoinsdbview.get()));
    int threads = opts.scriptThreads <= 0 ? GetNumCores() : opts.scriptThreads;
    threads = std::max(1, std::min(threads, MAX_SCRIPTCHECK_THREADS));
    pool.reset(new WorkerPool(threads));
    pcoinsTip->SetPool(pool.get()); // a block's view merges into the tip one shard per task
    scriptQueue.reset(new CheckQueue(threads - 1)); // the connecting thread is the last worker
    fReindex = opts.wipe;
}

Chainstate::~Chainstate() {
    if (g_chainstate == this) g_chainstate = nullptr;
}

void Chainstate::Shutdown() {
    std::lock_guard<CCriticalSection> l(cs_main);
    CValidationState state;
    FlushStateToDisk(state, FLUSH_STATE_ALWAYS);
}

CBlockIndex* Chainstate::LookupBlockIndex(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs_main); // callers outside cs_main too (RPC, net)
    auto it = mapBlockIndex.find(hash);
    return it == mapBlockIndex.end() ? nullptr : it->second;
}

CBlockIndex* Chainstate::InsertBlockIndex(const uint256& hash) {
    if (hash.IsNull()) return nullptr;
    auto it = mapBlockIndex.find(hash);
    if (it != mapBlockIndex.end()) return it->second;
    blockIndexStorage.emplace_back(new CBlockIndex());
    CBlockIndex* pindexNew = blockIndexStorage.back().get();
    auto ins = mapBlockIndex.emplace(hash, pindexNew);
    pindexNew->phashBlock = &ins.first->first;
    return pindexNew;
}

CBlockIndex* Chainstate::AddToBlockIndex(const CBlockHeader& block) {
    const uint256 hash = block.GetHash(params.GetConsensus());
    auto it = mapBlockIndex.find(hash);
    if (it != mapBlockIndex.end()) return it->second;
    blockIndexStorage.emplace_back(new CBlockIndex(block));
    CBlockIndex* pindexNew = blockIndexStorage.back().get();
    // BlockIndexes are only accessed under cs_main; sequence ids assigned on full data
    pindexNew->nSequenceId = 0;
    auto mi = mapBlockIndex.emplace(hash, pindexNew).first;
    pindexNew->phashBlock = &mi->first;
    auto miPrev = mapBlockIndex.find(block.hashPrevBlock);
    if (miPrev != mapBlockIndex.end()) {
        pindexNew->pprev = miPrev->second;
        pindexNew->nHeight = pindexNew->pprev->nHeight + 1;
        pindexNew->BuildSkip();
    }
    pindexNew->nTimeMax = pindexNew->pprev ? std::max(pindexNew->pprev->nTimeMax, pindexNew->nTime) : pindexNew->nTime;
    pindexNew->nChainWork = (pindexNew->pprev ? pindexNew->pprev->nChainWork : arith_uint256(0)) + GetBlockProof(*pindexNew);
    pindexNew->RaiseValidity(BLOCK_VALID_TREE);
    if (pindexBestHeader == nullptr || pindexBestHeader->nChainWork < pindexNew->nChainWork) pindexBestHeader = pindexNew;
    setDirtyBlockIndex.insert(pindexNew);
    return pindexNew;
}

// ------------------------------------------------------------------ checks
uint32_t Chainstate::GetBlockScriptFlags(const CBlockIndex* pindex) const {
    const Consensus::Params& cp = params.GetConsensus();
    const int64_t nBIP16SwitchTime = 1333238400;
    uint32_t flags = pindex->GetBlockTime() >= nBIP16SwitchTime ? SCRIPT_VERIFY_P2SH : SCRIPT_VERIFY_NONE;
    if (pindex->nHeight >= cp.BIP66Height) flags |= SCRIPT_VERIFY_DERSIG;
    if (pindex->nHeight >= cp.BIP65Height) flags |= SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY;
    if (VersionBitsState(pindex->pprev, cp, Consensus::DEPLOYMENT_CSV, const_cast<VersionBitsCache&>(versionbitscache)) ==
        THRESHOLD_ACTIVE)
        flags |= SCRIPT_VERIFY_CHECKSEQUENCEVERIFY;
    flags |= SCRIPT_ENABLE_SIGHASH_FORKID;
    if (IsBCPEnabled(pindex->pprev)) flags |= SCRIPT_VERIFY_STRICTENC | SCRIPT_VERIFY_LOW_S | SCRIPT_VERIFY_NULLFAIL;
    else flags |= SCRIPT_ALLOW_NON_FORKID;
    return flags;
}

bool Chainstate::CheckBlockHeader(const CBlockHeader& block, CValidationState& state, bool fCheckPOW) const {
    const bool postfork = IsBCPEnabled((int)block.nHeight);
    if (fCheckPOW && postfork && !CheckEquihashSolution(&block, params))
        return state.DoS(100, error("CheckBlockHeader(): Equihash solution invalid"), REJECT_INVALID,
                         "invalid-solution");
    if (fCheckPOW && !CheckProofOfWork(block.GetHash(params.GetConsensus()), block.nBits, postfork, params.GetConsensus()))
        return state.DoS(50, false, REJECT_INVALID, "high-hash", false, "proof of work failed");
    return true;
}

// GetSerializeSize(block, version) without walking the transactions again: each one's size was
// taken when its txid was hashed
uint64_t BlockSerializeSize(const CBlock& block, int version) {
    uint64_t n = GetSerializeSize(static_cast<const CBlockHeader&>(block), version) + GetSizeOfCompactSize(block.vtx.size());
    for (const auto& tx : block.vtx) n += tx->GetTotalSize();
    return n;
}

bool Chainstate::CheckBlock(const CBlock& block, CValidationState& state, bool fCheckPOW, bool fCheckMerkleRoot) const {
    if (block.fChecked) return true;
    if (!CheckBlockHeader(block, state, fCheckPOW)) return false;
    if (fCheckMerkleRoot) {
        bool mutated = false;
        const uint256 root = BlockMerkleRoot(block, &mutated);
        if (block.hashMerkleRoot != root)
            return state.DoS(100, false, REJECT_INVALID, "bad-txnmrklroot", true, "hashMerkleRoot mismatch");
        // CVE-2012-2459: a duplicated tail would give the same root
        if (mutated) return state.DoS(100, false, REJECT_INVALID, "bad-txns-duplicate", true, "duplicate transaction");
    }
    if (block.vtx.empty()) return state.DoS(100, false, REJECT_INVALID, "bad-cb-missing", false, "first tx is not coinbase");
    const int serFlags = IsBCPEnabled((int)block.nHeight) ? 0 : SERIALIZE_BLOCK_LEGACY;
    const uint64_t nMaxBlockSize = opts.maxBlockSize;
    if (block.vtx.size() * MIN_TRANSACTION_SIZE > nMaxBlockSize)
        return state.DoS(100, false, REJECT_INVALID, "bad-blk-length", false, "size limits failed");
    const uint64_t currentBlockSize = BlockSerializeSize(block, PROTOCOL_VERSION | serFlags);
    if (currentBlockSize > nMaxBlockSize)
        return state.DoS(100, false, REJECT_INVALID, "bad-blk-length", false, "size limits failed");
    if (!CheckCoinbase(*block.vtx[0], state, false))
        return state.Invalid(false, state.GetRejectCode(), state.GetRejectReason(),
                             strprintf("Coinbase check failed (txid %s) %s", block.vtx[0]->GetHash().ToString().c_str(),
                                       state.GetDebugMessage().c_str()));
    uint64_t nSigOps = 0;
    const uint64_t nMaxSigOpsCount = GetMaxBlockSigOpsCount(currentBlockSize);
    // Large blocks: the per-transaction checks run on the pool, then an in-order scan reports
    // the first failure exactly as the serial loop would (re-running that transaction's check
    // for its reject reason).
    const size_t ntx = block.vtx.size();
    std::vector<uint32_t> txSigOps;
    std::vector<uint8_t> txOk;
    if (pool && ntx >= 512) {
        txSigOps.resize(ntx);
        txOk.assign(ntx, 1);
        pool->ParallelFor(
            ntx,
            [&](size_t i) {
                const CTransaction& tx = *block.vtx[i];
                txSigOps[i] = (uint32_t)GetSigOpCountWithoutP2SH(tx);
                CValidationState st;
                if (i > 0 && !CheckRegularTransaction(tx, st, false)) txOk[i] = 0;
            },
            64);
    }
    for (size_t i = 0; i < ntx; i++) {
        const CTransaction& tx = *block.vtx[i];
        nSigOps += txSigOps.empty() ? GetSigOpCountWithoutP2SH(tx) : txSigOps[i];
        if (nSigOps > nMaxSigOpsCount)
            return state.DoS(100, false, REJECT_INVALID, "bad-blk-sigops", false, "out-of-bounds SigOpCount");
        if (i > 0 && (txOk.empty() || !txOk[i]) && !CheckRegularTransaction(tx, state, false))
            return state.Invalid(false, state.GetRejectCode(), state.GetRejectReason(),
                                 strprintf("Transaction check failed (txid %s) %s", tx.GetHash().ToString().c_str(),
                                           state.GetDebugMessage().c_str()));
    }
    if (fCheckPOW && fCheckMerkleRoot) block.fChecked = true;
    return true;
}

bool Chainstate::CheckIndexAgainstCheckpoint(const CBlockIndex* pindexPrev, CValidationState& state) const {
    if (*pindexPrev->phashBlock == params.GetConsensus().hashGenesisBlock) return true;
    const int nHeight = pindexPrev->nHeight + 1;
    // last checkpoint present in our index
    const auto& cps = params.Checkpoints().mapCheckpoints;
    for (auto it = cps.rbegin(); it != cps.rend(); ++it) {
        CBlockIndex* p = LookupBlockIndex(it->second);
        if (p) {
            if (nHeight < p->nHeight)
                return state.DoS(100, error("forked chain older than last checkpoint (height %d)", nHeight));
            break;
        }
    }
    return true;
}

bool Chainstate::ContextualCheckBlockHeader(const CBlockHeader& block, CValidationState& state,
                                            const CBlockIndex* pindexPrev, int64_t nAdjustedTime) const {
    const Consensus::Params& cp = params.GetConsensus();
    const int nHeight = pindexPrev == nullptr ? 0 : pindexPrev->nHeight + 1;
    if (block.nBits != GetNextWorkRequired(pindexPrev, &block, cp))
        return state.DoS(100, false, REJECT_INVALID, "bad-diffbits", false, "incorrect proof of work");
    if (IsBCPEnabled(nHeight) && block.nHeight != (uint32_t)nHeight)
        return state.Invalid(false, REJECT_INVALID, "bad-height", "incorrect block height");
    if (block.GetBlockTime() <= pindexPrev->GetMedianTimePast())
        return state.Invalid(false, REJECT_INVALID, "time-too-old", "block's timestamp is too early");
    if (block.GetBlockTime() > nAdjustedTime + 2 * 60 * 60)
        return state.Invalid(false, REJECT_INVALID, "time-too-new", "block timestamp too far in the future");
    if ((block.nVersion < 2 && nHeight >= cp.BIP34Height) || (block.nVersion < 3 && nHeight >= cp.BIP66Height) ||
        (block.nVersion < 4 && nHeight >= cp.BIP65Height))
        return state.Invalid(false, REJECT_OBSOLETE, strprintf("bad-version(0x%08x)", block.nVersion),
                             strprintf("rejected nVersion=0x%08x block", block.nVersion));
    return true;
}

bool Chainstate::ContextualCheckTransaction(const CTransaction& tx, CValidationState& state, int nHeight,
                                            int64_t nLockTimeCutoff) const {
    if (!IsFinalTx(tx, nHeight, nLockTimeCutoff))
        return state.DoS(10, false, REJECT_INVALID, "bad-txns-nonfinal", false, "non-final transaction");
    const Consensus::Params& cp = params.GetConsensus();
    if (IsBCPEnabled(nHeight) && nHeight <= cp.antiReplayOpReturnSunsetHeight) {
        for (const CTxOut& o : tx.vout)
            if (o.scriptPubKey.IsCommitment(cp.antiReplayOpReturnCommitment))
                return state.DoS(10, false, REJECT_INVALID, "bad-txn-replay", false, "non playable transaction");
    }
    return true;
}

bool Chainstate::ContextualCheckTransactionForCurrentBlock(const CTransaction& tx, CValidationState& state,
                                                           int flags) const {
    flags = std::max(flags, 0);
    const int nBlockHeight = chainActive.Height() + 1;
    const int64_t cutoff = (flags & LOCKTIME_MEDIAN_TIME_PAST) ? chainActive.Tip()->GetMedianTimePast() : GetAdjustedTime();
    return ContextualCheckTransaction(tx, state, nBlockHeight, cutoff);
}

bool Chainstate::ContextualCheckBlock(const CBlock& block, CValidationState& state, const CBlockIndex* pindexPrev) const {
    const Consensus::Params& cp = params.GetConsensus();
    const int nHeight = pindexPrev == nullptr ? 0 : pindexPrev->nHeight + 1;
    int nLockTimeFlags = 0;
    if (VersionBitsState(pindexPrev, cp, Consensus::DEPLOYMENT_CSV, const_cast<VersionBitsCache&>(versionbitscache)) ==
        THRESHOLD_ACTIVE)
        nLockTimeFlags |= LOCKTIME_MEDIAN_TIME_PAST;
    const int64_t nMedianTimePast = pindexPrev == nullptr ? 0 : pindexPrev->GetMedianTimePast();
    const int64_t cutoff = (nLockTimeFlags & LOCKTIME_MEDIAN_TIME_PAST) ? nMedianTimePast : block.GetBlockTime();
    for (const auto& tx : block.vtx)
        if (!ContextualCheckTransaction(*tx, state, nHeight, cutoff)) return false;
    if (nHeight >= cp.BIP34Height) {
        CScript expect = CScript() << nHeight;
        const CScript& sig = block.vtx[0]->vin[0].scriptSig;
        if (sig.size() < expect.size() || !std::equal(expect.begin(), expect.end(), sig.begin()))
            return state.DoS(100, false, REJECT_INVALID, "bad-cb-height", false, "block height mismatch in coinbase");
    }
    return true;
}

// ------------------------------------------------------------------ header / block acceptance
bool Chainstate::AcceptBlockHeader(const CBlockHeader& block, CValidationState& state, CBlockIndex** ppindex,
                                   bool equihashChecked) {
    const uint256 hash = block.GetHash(params.GetConsensus());
    CBlockIndex* pindex = nullptr;
    if (hash != params.GetConsensus().hashGenesisBlock) {
        auto miSelf = mapBlockIndex.find(hash);
        if (miSelf != mapBlockIndex.end()) {
            pindex = miSelf->second;
            if (ppindex) *ppindex = pindex;
            if (pindex->nStatus & BLOCK_FAILED_MASK)
                return state.Invalid(error("%s: block %s is marked invalid", __func__, hash.ToString().c_str()), 0,
                                     "duplicate");
            return true;
        }
        if (equihashChecked) {
            const bool postfork = IsBCPEnabled((int)block.nHeight);
            if (!CheckProofOfWork(hash, block.nBits, postfork, params.GetConsensus()))
                return state.DoS(50, false, REJECT_INVALID, "high-hash", false, "proof of work failed");
        } else if (!CheckBlockHeader(block, state)) {
            return error("%s: Consensus::CheckBlockHeader: %s, %s", __func__, hash.ToString().c_str(),
                         FormatStateMessage(state).c_str());
        }
        auto mi = mapBlockIndex.find(block.hashPrevBlock);
        if (mi == mapBlockIndex.end()) return state.DoS(10, error("%s: prev block not found", __func__), 0, "bad-prevblk");
        CBlockIndex* pindexPrev = mi->second;
        if (pindexPrev->nStatus & BLOCK_FAILED_MASK)
            return state.DoS(100, error("%s: prev block invalid", __func__), REJECT_INVALID, "bad-prevblk");
        if (opts.checkpoints && !CheckIndexAgainstCheckpoint(pindexPrev, state))
            return error("%s: CheckIndexAgainstCheckpoint(): %s", __func__, state.GetRejectReason().c_str());
        if (!ContextualCheckBlockHeader(block, state, pindexPrev, GetAdjustedTime()))
            return error("%s: Consensus::ContextualCheckBlockHeader: %s, %s", __func__, hash.ToString().c_str(),
                         FormatStateMessage(state).c_str());
    }
    if (pindex == nullptr) pindex = AddToBlockIndex(block);
    if (ppindex) *ppindex = pindex;
    CheckBlockIndex();
    return true;
}

void Chainstate::NotifyHeaderTip() {
    static CBlockIndex* pindexHeaderOld = nullptr;
    CBlockIndex* pindexHeader = nullptr;
    bool fNotify = false, ibd = false;
    {
        std::lock_guard<CCriticalSection> l(cs_main);
        pindexHeader = pindexBestHeader;
        if (pindexHeader != pindexHeaderOld) {
            fNotify = true;
            ibd = IsInitialBlockDownload();
            pindexHeaderOld = pindexHeader;
        }
    }
    if (fNotify) {
        GetMainSignals().NotifyHeaderTip(pindexHeader, ibd);
        uiInterface.NotifyHeaderTip(ibd, pindexHeader);
    }
}

bool Chainstate::ProcessNewBlockHeaders(const std::vector<CBlockHeader>& headers, CValidationState& state,
                                        const CBlockIndex** ppindex) {
    // Batch the Equihash checks of unknown post-fork headers (GPU when >= 4 headers).
    std::vector<const CBlockHeader*> toCheck;
    std::vector<size_t> pos;
    {
        std::lock_guard<CCriticalSection> l(cs_main);
        for (size_t i = 0; i < headers.size(); i++) {
            if (!IsBCPEnabled((int)headers[i].nHeight)) continue;
            if (mapBlockIndex.count(headers[i].GetHash(params.GetConsensus()))) continue;
            toCheck.push_back(&headers[i]);
            pos.push_back(i);
        }
    }
    std::vector<bool> eqOk(headers.size(), true);
    if (!toCheck.empty()) {
        std::vector<bool> r = CheckEquihashSolutions(toCheck, params, opts.useGpu);
        for (size_t j = 0; j < r.size(); j++) eqOk[pos[j]] = r[j];
    }
    {
        std::lock_guard<CCriticalSection> l(cs_main);
        for (size_t i = 0; i < headers.size(); i++) {
            if (!eqOk[i])
                return state.DoS(100, error("ProcessNewBlockHeaders(): Equihash solution invalid"), REJECT_INVALID,
                                 "invalid-solution");
            CBlockIndex* pindex = nullptr;
            if (!AcceptBlockHeader(headers[i], state, &pindex, IsBCPEnabled((int)headers[i].nHeight))) return false;
            if (ppindex) *ppindex = pindex;
        }
    }
    NotifyHeaderTip();
    return true;
}

bool Chainstate::FindBlockPos(CValidationState& state, CDiskBlockPos& pos, unsigned nAddSize, unsigned nHeight,
                              uint64_t nTime, bool fKnown) {
    unsigned nFile = fKnown ? pos.nFile : nLastBlockFile;
    if (vinfoBlockFile.size() <= nFile) vinfoBlockFile.resize(nFile + 1);
    if (!fKnown) {
        while (vinfoBlockFile[nFile].nSize + nAddSize >= FileSizes().maxFile) {
            nFile++;
            if (vinfoBlockFile.size() <= nFile) vinfoBlockFile.resize(nFile + 1);
        }
        pos.nFile = nFile;
        pos.nPos = vinfoBlockFile[nFile].nSize;
    }
    if ((int)nFile != nLastBlockFile) {
        if (!fKnown) LogPrintf("Leaving block file %i: %s\n", nLastBlockFile, vinfoBlockFile[nLastBlockFile].ToString().c_str());
        FlushBlockFile(!fKnown);
        nLastBlockFile = nFile;
    }
    vinfoBlockFile[nFile].AddBlock(nHeight, nTime);
    if (fKnown) vinfoBlockFile[nFile].nSize = std::max(pos.nPos + nAddSize, vinfoBlockFile[nFile].nSize);
    else vinfoBlockFile[nFile].nSize += nAddSize;
    if (!fKnown) {
        const unsigned chunk = FileSizes().blockChunk;
        const unsigned nOldChunks = (pos.nPos + chunk - 1) / chunk;
        const unsigned nNewChunks = (vinfoBlockFile[nFile].nSize + chunk - 1) / chunk;
        if (nNewChunks > nOldChunks) {
            if (PruneMode()) fCheckForPruning = true;
            FILE* file = OpenBlockFile(pos);
            if (file) {
                AllocateFileRange(file, pos.nPos, nNewChunks * chunk - pos.nPos);
                fclose(file);
            } else {
                return state.Error("out of disk space");
            }
        }
    }
    setDirtyFileInfo.insert(nFile);
    return true;
}

bool Chainstate::FindUndoPos(CValidationState& state, int nFile, CDiskBlockPos& pos, unsigned nAddSize) {
    pos.nFile = nFile;
    const unsigned nNewSize = vinfoBlockFile[nFile].nUndoSize += nAddSize;
    pos.nPos = nNewSize - nAddSize;
    setDirtyFileInfo.insert(nFile);
    const unsigned chunk = FileSizes().undoChunk;
    const unsigned nOldChunks = (pos.nPos + chunk - 1) / chunk;
    const unsigned nNewChunks = (nNewSize + chunk - 1) / chunk;
    if (nNewChunks > nOldChunks) {
        if (PruneMode()) fCheckForPruning = true;
        FILE* file = OpenUndoFile(pos);
        if (!file) return state.Error("out of disk space");
        AllocateFileRange(file, pos.nPos, nNewChunks * chunk - pos.nPos);
        fclose(file);
    }
    return true;
}

void Chainstate::FlushBlockFile(bool fFinalize) {
    CDiskBlockPos posOld(nLastBlockFile, 0);
    if (FILE* f = OpenBlockFile(posOld)) {
        if (fFinalize && nLastBlockFile < (int)vinfoBlockFile.size() &&
            ftruncate(fileno(f), vinfoBlockFile[nLastBlockFile].nSize) != 0) {
        }
        FileCommit(f);
        fclose(f);
    }
    if (FILE* f = OpenUndoFile(posOld)) {
        if (fFinalize && nLastBlockFile < (int)vinfoBlockFile.size() &&
            ftruncate(fileno(f), vinfoBlockFile[nLastBlockFile].nUndoSize) != 0) {
        }
        FileCommit(f);
        fclose(f);
    }
}

bool Chainstate::ReceivedBlockTransactions(const CBlock& block, CValidationState& state, CBlockIndex* pindexNew,
                                           const CDiskBlockPos& pos) {
    pindexNew->nTx = (unsigned)block.vtx.size();
    pindexNew->nChainTx = 0;
    pindexNew->nFile = pos.nFile;
    pindexNew->nDataPos = pos.nPos;
    pindexNew->nUndoPos = 0;
    pindexNew->nStatus |= BLOCK_HAVE_DATA;
    pindexNew->RaiseValidity(BLOCK_VALID_TRANSACTIONS);
    setDirtyBlockIndex.insert(pindexNew);
    if (pindexNew->pprev == nullptr || pindexNew->pprev->nChainTx) {
        // the block and all its descendants waiting for data can now be linked
        std::deque<CBlockIndex*> queue;
        queue.push_back(pindexNew);
        while (!queue.empty()) {
            CBlockIndex* pindex = queue.front();
            queue.pop_front();
            pindex->nChainTx = (pindex->pprev ? pindex->pprev->nChainTx : 0) + pindex->nTx;
            pindex->nSequenceId = nBlockSequenceId++;
            if (chainActive.Tip() == nullptr || !setBlockIndexCandidates.value_comp()(pindex, chainActive.Tip()))
                setBlockIndexCandidates.insert(pindex);
            auto range = mapBlocksUnlinked.equal_range(pindex);
            while (range.first != range.second) {
                queue.push_back(range.first->second);
                range.first = mapBlocksUnlinked.erase(range.first);
            }
        }
    } else if (pindexNew->pprev && pindexNew->pprev->IsValid(BLOCK_VALID_TREE)) {
        mapBlocksUnlinked.insert(std::make_pair(pindexNew->pprev, pindexNew));
    }
    return true;
}

bool Chainstate::AcceptBlock(const std::shared_ptr<const CBlock>& pblock, CValidationState& state, CBlockIndex** ppindex,
                             bool fRequested, const CDiskBlockPos* dbp, bool* fNewBlock) {
    const CBlock& block = *pblock;
    if (fNewBlock) *fNewBlock = false;
    CBlockIndex* pindexDummy = nullptr;
    CBlockIndex*& pindex = ppindex ? *ppindex : pindexDummy;
    if (!AcceptBlockHeader(block, state, &pindex)) return false;
    const bool fAlreadyHave = pindex->nStatus & BLOCK_HAVE_DATA;
    const bool fHasMoreWork = chainActive.Tip() ? pindex->nChainWork > chainActive.Tip()->nChainWork : true;
    const bool fTooFarAhead = pindex->nHeight > int(chainActive.Height() + MIN_BLOCKS_TO_KEEP);
    if (fAlreadyHave) return true;
    if (!fRequested) {
        if (pindex->nTx != 0) return true;
        if (!fHasMoreWork) return true;
        if (fTooFarAhead) return true;
    }
    if (fNewBlock) *fNewBlock = true;
    if (!CheckBlock(block, state) || !ContextualCheckBlock(block, state, pindex->pprev)) {
        if (state.IsInvalid() && !state.CorruptionPossible()) {
            pindex->nStatus |= BLOCK_FAILED_VALID;
            setDirtyBlockIndex.insert(pindex);
        }
        return error("%s: %s (block %s)", __func__, FormatStateMessage(state).c_str(),
                     block.GetHash(params.GetConsensus()).ToString().c_str());
    }
    if (!IsInitialBlockDownload() && chainActive.Tip() == pindex->pprev) GetMainSignals().NewPoWValidBlock(pindex, pblock);
    const int nHeight = pindex->nHeight;
    try {
        const unsigned nBlockSize = (unsigned)BlockSerializeSize(block, PROTOCOL_VERSION);
        CDiskBlockPos blockPos;
        if (dbp != nullptr) blockPos = *dbp;
        if (!FindBlockPos(state, blockPos, nBlockSize + 8, nHeight, block.GetBlockTime(), dbp != nullptr))
            return error("AcceptBlock(): FindBlockPos failed");
        if (dbp == nullptr && !WriteBlockToDisk(block, blockPos, params.DiskMagic()))
            return state.Error("Failed to write block");
        if (!ReceivedBlockTransactions(block, state, pindex, blockPos))
            return error("AcceptBlock(): ReceivedBlockTransactions failed");
        // kept until it connects (ActivateBestChain hands ConnectTip only the block it was
        // called with; every other block of the step would be read back from disk)
        CacheRecentBlock(pindex->GetBlockHash(), pblock, nBlockSize);
    } catch (const std::runtime_error& e) {
        return state.Error(std::string("System error: ") + e.what());
    }
    if (fCheckForPruning) FlushStateToDisk(state, FLUSH_STATE_NONE);
    return true;
}

// Heap bytes a decoded block holds (the transactions, their input/output vectors and scripts,
// the shared_ptr control blocks): several times its serialized size, and what -blockcachemb
// counts.
static size_t BlockMemoryUsage(const CBlock& block) {
    size_t m = memusage::DynamicUsage(block.vtx);
    for (const CTransactionRef& tx : block.vtx) {
        m += memusage::MallocUsage(sizeof(CTransaction) + 16); // object + control block (make_shared)
        m += memusage::DynamicUsage(tx->vin) + memusage::DynamicUsage(tx->vout);
        for (const CTxIn& in : tx->vin) m += memusage::DynamicUsage(static_cast<const CScriptBase&>(in.scriptSig));
        for (const CTxOut& out : tx->vout)
            m += memusage::DynamicUsage(static_cast<const CScriptBase&>(out.scriptPubKey));
    }
    return m;
}

void Chainstate::CacheRecentBlock(const uint256& hash, const std::shared_ptr<const CBlock>& pblock, size_t) {
    const size_t bytes = BlockMemoryUsage(*pblock);
    if (bytes > opts.recentBlockBytes || recentBlocks.count(hash)) return;
    while (recentBytes + bytes > opts.recentBlockBytes && !recentOrder.empty()) {
        auto it = recentBlocks.find(recentOrder.front());
        recentOrder.pop_front();
        if (it == recentBlocks.end()) continue; // taken already
        recentBytes -= it->second.second;
        recentBlocks.erase(it);
    }
    recentBlocks.emplace(hash, std::make_pair(pblock, bytes));
    recentOrder.push_back(hash);
    recentBytes += bytes;
}

std::shared_ptr<const CBlock> Chainstate::TakeRecentBlock(const uint256& hash) {
    auto it = recentBlocks.find(hash);
    if (it == recentBlocks.end()) return nullptr;
    std::shared_ptr<const CBlock> b = std::move(it->second.first);
    recentBytes -= it->second.second;
    recentBlocks.erase(it);
    // taken blocks leave their hash in the eviction order; drop those once they outnumber the
    // cached blocks (a stale-fork block that never connects keeps the map non-empty forever)
    if (recentOrder.size() > 2 * recentBlocks.size() + 64) {
        std::deque<uint256> keep;
        for (const uint256& h : recentOrder)
            if (recentBlocks.count(h)) keep.push_back(h);
        recentOrder.swap(keep);
    }
    return b;
}

bool Chainstate::ProcessNewBlock(const std::shared_ptr<const CBlock>& pblock, bool fForceProcessing, bool* fNewBlock,
                                 CValidationState* stateOut) {
    {
        CBlockIndex* pindex = nullptr;
        if (fNewBlock) *fNewBlock = false;
        CValidationState state;
        const int64_t tAccept = GetTimeMicros();
        // the expensive context-free checks (Equihash, merkle) run before taking cs_main
        bool ret = CheckBlock(*pblock, state);
        std::lock_guard<CCriticalSection> l(cs_main);
        if (ret) ret = AcceptBlock(pblock, state, &pindex, fForceProcessing, nullptr, fNewBlock);
        CheckBlockIndex();
        phaseMicros[PH_ACCEPT].fetch_add(GetTimeMicros() - tAccept, std::memory_order_relaxed);
        if (!ret) {
            GetMainSignals().BlockChecked(*pblock, state);
            if (stateOut) *stateOut = state;
            return error("%s: AcceptBlock FAILED (%s)", __func__, FormatStateMessage(state).c_str());
        }
    }
    NotifyHeaderTip();
    CValidationState state;
    if (!ActivateBestChain(state, pblock)) {
        if (stateOut) *stateOut = state;
        return error("%s: ActivateBestChain failed (%s)", __func__, FormatStateMessage(state).c_str());
    }
    if (stateOut) *stateOut = state;
    return true;
}

bool Chainstate::TestBlockValidity(CValidationState& state, const CBlock& block, CBlockIndex* pindexPrev, bool fCheckPOW,
                                   bool fCheckMerkleRoot) {
    std::lock_guard<CCriticalSection> l(cs_main);
    if (!(pindexPrev && pindexPrev == chainActive.Tip())) return state.Error("TestBlockValidity: not on tip");
    // the block's coins view is freed on the reaper thread (util/reaper.h)
    std::unique_ptr<CCoinsViewCache> viewNew(new CCoinsViewCache(pcoinsTip.get()));
    struct DropView {
        std::unique_ptr<CCoinsViewCache>& v;
        ~DropView() { Reaper::Get().Drop(std::move(v)); }
    } dropView{viewNew};
    CBlockIndex indexDummy(block);
    indexDummy.pprev = pindexPrev;
    indexDummy.nHeight = pindexPrev->nHeight + 1;
    if (!ContextualCheckBlockHeader(block, state, pindexPrev, GetAdjustedTime()))
        return error("%s: Consensus::ContextualCheckBlockHeader: %s", __func__, FormatStateMessage(state).c_str());
    if (!CheckBlock(block, state, fCheckPOW, fCheckMerkleRoot))
        return error("%s: Consensus::CheckBlock: %s", __func__, FormatStateMessage(state).c_str());
    if (!ContextualCheckBlock(block, state, pindexPrev))
        return error("%s: Consensus::ContextualCheckBlock: %s", __func__, FormatStateMessage(state).c_str());
    if (!ConnectBlock(block, state, &indexDummy, *viewNew, true)) return false;
    return true;
}

// ------------------------------------------------------------------ connect / disconnect
bool Chainstate::CheckInputs(const CTransaction& tx, CValidationState& state, const CCoinsViewCache& inputs,
                             bool fScriptChecks, uint32_t flags, bool cacheStore,
                             const PrecomputedTransactionData& txdata) {
    // mempool path: eager evaluation with the caching checker (block path is batched in ConnectBlock)
    if (!Consensus::CheckTxInputs(tx, state, inputs, chainActive.Height() + 1)) return false;
    if (!fScriptChecks) return true;
    ScriptCache& sc = GetScriptCache();
    const uint256 key = sc.Key(tx, flags);
    if (sc.Has(key, false)) return true;
    for (size_t i = 0; i < tx.vin.size(); i++) {
        const Coin& coin = inputs.AccessCoin(tx.vin[i].prevout);
        const CScript& spk = coin.GetTxOut().scriptPubKey;
        const Amount amount = coin.GetTxOut().nValue;
        ScriptError err;
        CachingTransactionSignatureChecker checker(&tx, (unsigned)i, amount, cacheStore, &txdata);
        if (!VerifyScript(tx.vin[i].scriptSig, spk, flags, checker, &err)) {
            if (flags & STANDARD_NOT_MANDATORY_VERIFY_FLAGS) {
                ScriptError err2;
                CachingTransactionSignatureChecker checker2(&tx, (unsigned)i, amount, cacheStore, &txdata);
                if (VerifyScript(tx.vin[i].scriptSig, spk, flags & ~STANDARD_NOT_MANDATORY_VERIFY_FLAGS, checker2, &err2))
                    return state.Invalid(false, REJECT_NONSTANDARD,
                                         strprintf("non-mandatory-script-verify-flag (%s)", ScriptErrorString(err)));
            }
            return state.DoS(100, false, REJECT_INVALID,
                             strprintf("mandatory-script-verify-flag-failed (%s)", ScriptErrorString(err)));
        }
    }
    if (cacheStore) sc.Add(key);
    return true;
}

struct Chainstate::PendingConnect {
    CBlockIndex* pindex = nullptr;
    bool genesis = false, postfork = false;
    size_t nJobs = 0;               // script jobs run for this block
    bool sigsOk = true;             // the batch's verdict (false too when scripts failed)
    CBlockUndo blockundo;
    std::vector<std::pair<uint256, CDiskTxPos>> vPos;
    int64_t nTimeStart = 0, nTime2 = 0;
    int nInputs = 0;
    // The coins tip under the (empty) view, when the caller lets the parallel UTXO pass update
    // it in place instead of the view (ConnectTip); `tipApplied` once it did, so that a verdict
    // that fails afterwards undoes the block on the tip from its undo records.
    CCoinsViewCache* directTip = nullptr;
    bool tipApplied = false;
    // the undo record serialised and checksummed on a helper thread while the signature batch
    // runs on the GPU (joined before blockundo may move or die)
    std::future<std::pair<std::vector<unsigned char>, uint256>> undoSer;
};

namespace {
// Appends to a byte vector with amortised doubling and memcpy (VectorWriter's per-field
// vector::insert dominates a 40k-coin undo record's serialisation).
class FastVectorWriter {
public:
    explicit FastVectorWriter(std::vector<unsigned char>& out) : v(out), len(out.size()) {}
    ~FastVectorWriter() { v.resize(len); }
    int GetType() const { return SER_DISK; }
    int GetVersion() const { return PROTOCOL_VERSION; }
    void write(const char* p, size_t k) {
        if (len + k > v.size()) v.resize(std::max<size_t>(2 * v.size(), len + k + 4096));
        memcpy(v.data() + len, p, k);
        len += k;
    }
    template <typename T> FastVectorWriter& operator<<(const T& obj) {
        ::bcp::Serialize(*this, obj);
        return *this;
    }

private:
    std::vector<unsigned char>& v;
    size_t len;
};
} // namespace

// The block's undo record in its disk (SER_DISK) serialisation, transaction chunks serialised in
// parallel and concatenated (the same bytes as SerializeToBytes(undo): CompactSize count, then
// each CTxUndo in order). A 21k-transaction block's record is ~1.1 MB of small varint fields.
std::vector<unsigned char> SerializeBlockUndo(const CBlockUndo& undo, WorkerPool* pool) {
    const size_t n = undo.vtxundo.size();
    std::vector<unsigned char> out;
    const bool serial = !pool || n < 1024;
    {
        // the writer trims `out` to what it wrote when it goes out of scope: return only after
        FastVectorWriter w(out);
        WriteCompactSize(w, n);
        if (serial)
            for (const CTxUndo& u : undo.vtxundo) w << u;
    }
    if (serial) return out;
    const size_t chunks = std::min<size_t>(64, n / 256);
    std::vector<std::vector<unsigned char>> parts(chunks);
    pool->ParallelFor(chunks, [&](size_t c) {
        const size_t lo = n * c / chunks, hi = n * (c + 1) / chunks;
        parts[c].resize((hi - lo) * 72);
        parts[c].clear(); // keeps the capacity; the writer grows the size as it goes
        FastVectorWriter w(parts[c]);
        for (size_t i = lo; i < hi; i++) w << undo.vtxundo[i];
    });
    size_t total = out.size();
    for (const auto& p : parts) total += p.size();
    out.reserve(total);
    for (const auto& p : parts) out.insert(out.end(), p.begin(), p.end());
    return out;
}

// BIP30 exceptions: the two historic duplicate coinbases
static bool IsBIP30Exception(const CBlockIndex* pindex) {
    return pindex->phashBlock &&
           ((pindex->nHeight == 91842 &&
             pindex->GetBlockHash() == uint256S("0x00000000000a4d0a398161ffc163c503763b1f4360639393e0e4c8e300e0caec")) ||
            (pindex->nHeight == 91880 &&
             pindex->GetBlockHash() == uint256S("0x00000000000743f190a18c5577a3c2d2a1f610ae9601ac046a38084ccb7cd721")));
}

// BIP30 is checked except for the two exceptions and after the BIP34 block (reference
// validation.cpp:1952-1980)
bool Chainstate::EnforceBIP30For(const CBlockIndex* pindex) const {
    const Consensus::Params& cp = params.GetConsensus();
    const CBlockIndex* pindexBIP34height = pindex->pprev->GetAncestor(cp.BIP34Height);
    return !IsBIP30Exception(pindex) && (!pindexBIP34height || !(pindexBIP34height->GetBlockHash() == cp.BIP34Hash));
}

// -assumevalid: scripts are skipped for an ancestor of the assumed-valid block that is buried
// under two weeks of work below the best header (reference validation.cpp:1925-1948)
bool Chainstate::ScriptChecksFor(const CBlockIndex* pindex) const {
    if (opts.assumeValid.IsNull()) return true;
    const Consensus::Params& cp = params.GetConsensus();
    auto it = mapBlockIndex.find(opts.assumeValid);
    if (it != mapBlockIndex.end() && it->second->GetAncestor(pindex->nHeight) == pindex && pindexBestHeader &&
        pindexBestHeader->GetAncestor(pindex->nHeight) == pindex &&
        pindexBestHeader->nChainWork >= UintToArith256(cp.nMinimumChainWork))
        return GetBlockProofEquivalentTime(*pindexBestHeader, *pindex, *pindexBestHeader, cp) <= 60 * 60 * 24 * 7 * 2;
    return true;
}

std::shared_ptr<const CBlock> Chainstate::PeekRecentBlock(const uint256& hash) const {
    auto it = recentBlocks.find(hash);
    return it == recentBlocks.end() ? nullptr : it->second.first;
}

// Called by block N's connect once its UTXO pass has updated the coins tip in place and its
// signatures are about to go to the GPU: block N+1 (the next block ActivateBestChainStep will
// connect, if it is in the recent-block cache) gets its read-only pass on the script threads,
// which are idle until N+1's scripts. Every coin it fetches is read from the tip as N left it.
void Chainstate::StartLookahead(const CBlockIndex* pindex) {
    lookahead.reset();
    const CBlockIndex* next = pindexConnectNext;
    if (!next || next->pprev != pindex) return;
    std::shared_ptr<const CBlock> nb = PeekRecentBlock(next->GetBlockHash());
    if (!nb || nb->vtx.size() < 1024) return;
    std::unique_ptr<Lookahead> la(new Lookahead());
    la->forHash = next->GetBlockHash();
    la->afterHash = pindex->GetBlockHash();
    la->pf.hold = nb;
    la->pf.Init(*nb, *pcoinsTip, EnforceBIP30For(next), ScriptChecksFor(next), GetScriptCache().MayHold(),
                GetBlockScriptFlags(next));
    Lookahead* raw = la.get();
    scriptQueue->Begin([raw](size_t k) { raw->pf.Job(k, GetScriptCache()); });
    scriptQueue->Publish(raw->pf.Jobs());
    la->open = true;
    lookahead = std::move(la);
}

// Closes the lookahead's script-queue session (this thread runs what is left of it). Must run
// before anything writes the coins tip or opens another session on the queue.
void Chainstate::JoinLookahead() {
    if (!lookahead || !lookahead->open) return;
    const int64_t t = GetTimeMicros();
    scriptQueue->Complete();
    lookahead->open = false;
    phaseMicros[PH_LA_WAIT].fetch_add(GetTimeMicros() - t, std::memory_order_relaxed);
}

bool Chainstate::ConnectBlock(const CBlock& block, CValidationState& state, CBlockIndex* pindex, CCoinsViewCache& view,
                              bool fJustCheck, CCoinsViewCache* directTip) {
    PendingConnect p;
    p.directTip = fJustCheck ? nullptr : directTip;
    bool ok = false;
    try {
        ok = ConnectBlockPrepare(block, state, pindex, view, fJustCheck, p) && ConnectBlockFinish(p, state, fJustCheck);
    } catch (...) {
        JoinLookahead();
        lookahead.reset();
        if (p.undoSer.valid()) p.undoSer.wait();
        throw;
    }
    // the lookahead for the next block ran through the verdict and the undo write; it read the
    // tip as this block left it, so it goes if this block is taken back off the tip
    JoinLookahead();
    if (!ok) lookahead.reset();
    if (p.undoSer.valid()) p.undoSer.wait(); // it reads blockundo
    if (!ok && p.tipApplied) {
        // a verdict after the in-place update failed: take the block back off the tip (its outputs
        // removed, the spent coins restored from the undo records), as DisconnectBlock would
        if (ApplyBlockUndo(p.blockundo, block, pindex, *p.directTip) != DISCONNECT_OK)
            LogPrintf("ConnectBlock: undoing the failed block %s on the coins tip was not clean\n",
                      pindex->GetBlockHash().ToString().c_str());
    }
    Reaper::Get().Drop(std::move(p.blockundo)); // 21k+ undo vectors for a big block
    return ok;
}

// Phase 1 of connecting a block: every consensus check that needs the UTXO view, the script
// runs (ECDSA deferred) and the block's signature batch. The view (or, in place, the tip) is
// fully updated when this returns; the block is valid only once Finish agrees.
bool Chainstate::ConnectBlockPrepare(const CBlock& block, CValidationState& state, CBlockIndex* pindex,
                                     CCoinsViewCache& view, bool fJustCheck, PendingConnect& p) {
    JoinLookahead(); // normally closed already (ConnectBlock joins it after the previous block)
    const int64_t nTimeStart = GetTimeMicros();
    p.pindex = pindex;
    p.nTimeStart = nTimeStart;
    const Consensus::Params& cp = params.GetConsensus();
    if (!CheckBlock(block, state, !fJustCheck, !fJustCheck))
        return error("%s: Consensus::CheckBlock: %s", __func__, FormatStateMessage(state).c_str());
    int64_t tPhase = nTimeStart;
    auto phase = [&](ConnectPhase ph) {
        const int64_t t = GetTimeMicros();
        phaseMicros[ph].fetch_add(t - tPhase, std::memory_order_relaxed);
        tPhase = t;
    };
    phase(PH_CHECK);
    phaseMicros[PH_BLOCKS].fetch_add(1, std::memory_order_relaxed);
    const uint256 hashPrevBlock = pindex->pprev == nullptr ? uint256() : pindex->pprev->GetBlockHash();
    if (hashPrevBlock != view.GetBestBlock()) return state.Error("ConnectBlock: view best block mismatch");
    if (block.GetHash(cp) == cp.hashGenesisBlock) {
        if (!fJustCheck) view.SetBestBlock(pindex->GetBlockHash());
        p.genesis = true;
        return true;
    }
    const bool fScriptChecks = ScriptChecksFor(pindex);
    const bool fBIP30Exception = IsBIP30Exception(pindex);
    const bool fEnforceBIP30 = EnforceBIP30For(pindex);
    int nLockTimeFlags = 0;
    if (VersionBitsState(pindex->pprev, cp, Consensus::DEPLOYMENT_CSV, versionbitscache) == THRESHOLD_ACTIVE)
        nLockTimeFlags |= LOCKTIME_VERIFY_SEQUENCE;
    const uint32_t flags = GetBlockScriptFlags(pindex);
    const bool postfork = IsBCPEnabled(pindex->nHeight);

    CBlockUndo& blockundo = p.blockundo;
    std::vector<int> prevheights;
    Amount nFees = 0;
    int nInputs = 0;
    uint64_t nSigOpsCount = 0;
    const uint64_t currentBlockSize = BlockSerializeSize(block, PROTOCOL_VERSION); // cached tx sizes, no re-walk
    const uint64_t nMaxSigOpsCount = GetMaxBlockSigOpsCount(currentBlockSize);
    CDiskTxPos pos(pindex->GetBlockPos(), GetSizeOfCompactSize(block.vtx.size()));
    std::vector<std::pair<uint256, CDiskTxPos>>& vPos = p.vPos;
    vPos.reserve(block.vtx.size());
    blockundo.vtxundo.reserve(block.vtx.size() - 1);
    const size_t ntx = block.vtx.size();
    ScriptCache& sc = GetScriptCache();
    // ConnectBlock only reads the script cache (mempool acceptance fills it, under cs_main as
    // this is): while it was never filled every lookup would miss, so no key is computed
    const bool scMayHold = sc.MayHold();

    // One parallel, read-only pass over the block before anything writes the view stack
    // (BlockPrefetch): so the UTXO pass below inserts each input's coin into the view instead of
    // walking the view stack itself - a coin created or spent earlier in this block is found in
    // the view first, so the prefetched copy of an outpoint is only used while it is still
    // current. The previous block's connect may have run it already (the lookahead): adopted
    // when it is this block's, read the tip as it is now, and under this block's flags.
    std::unique_ptr<Lookahead> la = std::move(lookahead);
    std::unique_ptr<BlockPrefetch> own;
    BlockPrefetch* pf = nullptr;
    if (la && !fJustCheck && la->forHash == pindex->GetBlockHash() && la->afterHash == hashPrevBlock &&
        view.GetCacheSize() == 0 && la->pf.ntx == ntx && la->pf.flags == flags &&
        la->pf.fEnforceBIP30 == fEnforceBIP30 && la->pf.fScriptChecks == fScriptChecks && la->pf.scMayHold == scMayHold) {
        pf = &la->pf;
        phaseMicros[PH_LA_USED].fetch_add(1, std::memory_order_relaxed);
    } else {
        own.reset(new BlockPrefetch());
        own->Init(block, view, fEnforceBIP30, fScriptChecks, scMayHold, flags);
        pool->ParallelFor(own->Jobs(), [&](size_t k) { own->Job(k, sc); }, 1);
        pf = own.get();
    }
    std::vector<std::unique_ptr<PrecomputedTransactionData>>& txdatas = pf->txdatas;
    const std::vector<uint256>& scKeys = pf->scKeys;
    const std::vector<uint32_t>& txSizes = pf->txSizes;
    const std::vector<uint32_t>& legacySigOps = pf->legacySigOps;
    const std::vector<size_t>& firstInput = pf->firstInput;
    std::vector<Coin>& prefetched = pf->prefetched;
    const std::unique_ptr<uint8_t[]>& prefetchedFound = pf->prefetchedFound;
    const size_t nOutputs = pf->nOutputs, maxJobs = pf->maxJobs;
    if (pf->bip30Clash)
        return state.DoS(100, error("ConnectBlock(): tried to overwrite transaction"), REJECT_INVALID, "bad-txns-BIP30");
    phase(PH_PRECOMPUTE);

    // Script checks overlap the UTXO pass (reference CCheckQueue: the master keeps connecting
    // while workers run the queued CScriptChecks, src/validation.cpp:2011-2127). The loop below
    // publishes jobs into a pre-sized array; the script queue's own threads execute them as they
    // appear (sleeping while none are available), deferring every ECDSA check into a per-job sink
    // for the batch verifier. Nothing in the UTXO loop may wait on the queue's threads.
    // coins of in-block outputs spent within the block (and copies of the view's own coins): the
    // parallel pass's script jobs read them, so they outlive the script session (declared before
    // completeOnExit, which closes it)
    // (one deque per chunk of transactions: stable addresses, filled only for the rare inputs
    // that need one, no per-input array to construct)
    std::vector<std::deque<Coin>> made;
    std::vector<ScriptJob> jobs(maxJobs);
    std::vector<std::vector<DeferredSigCheck>> sinks(maxJobs);
    std::vector<std::vector<DeferredMultisig>> groupSinks(maxJobs); // deferred CHECKMULTISIGs per job
    const bool deferMultisig = GpuBatchesExpected(opts.useGpu);
    std::atomic<bool> anyFail{false};
    size_t nProduced = 0, nPublished = 0;
    const bool queued = fScriptChecks && maxJobs > 0;
    if (queued)
        scriptQueue->Begin([&](size_t k) {
            if (anyFail.load(std::memory_order_relaxed)) return;
            const ScriptJob& J = jobs[k];
            BlockSigChecker checker(J.tx, J.nIn, J.amount, J.txdata, &sinks[k], deferMultisig ? &groupSinks[k] : nullptr);
            ScriptError err;
            if (!VerifyScript(J.tx->vin[J.nIn].scriptSig, *J.scriptPubKey, flags, checker, &err)) anyFail = true;
        });
    // every return below drains and closes the session first (jobs/sinks outlive it)
    struct CompleteOnExit {
        CheckQueue& q;
        bool armed = true;
        ~CompleteOnExit() {
            if (armed) q.Complete();
        }
    } completeOnExit{*scriptQueue};

    // The UTXO pass, in parallel for a valid block (round 4). Every input's coin is resolved
    // without touching the view: the view's own entry, else an output of an earlier transaction
    // of this block (block-local txid index), else the prefetched coin. All per-transaction checks
    // (missing or doubly spent inputs, BIP68, sigop limits, amounts, coinbase maturity) run on the
    // pool; the block sigop total is a prefix sum. Only a block that passes everything takes the
    // fast path: undo records and script jobs are built in parallel, the scripts start, and the
    // view is then updated serially while they run - spends of fetched coins, spends of the view's
    // own coins, and the outputs that no later transaction of the block spends (an output created
    // and spent inside the block leaves no entry, as AddCoin + SpendCoin of a FRESH entry would).
    // Any failure, or an unusual overlap of the view with the block's own outputs, runs the
    // serial pass below instead, which yields the reference's exact reject reason.
    bool fastDone = false;
    // Taken whenever the block is not one of the two historic BIP30 exceptions: with BIP30
    // enforced the prefetch above has checked every output; after the BIP34 block txids are
    // unique and, like the serial pass's AddCoins, the output adds assume no overwrite.
    if (!fBIP30Exception && opts.parallelUtxoMinTx > 0 && ntx >= opts.parallelUtxoMinTx && maxJobs > 0) {
        int64_t tSub = GetTimeMicros();
        auto sub = [&](ConnectPhase ph) {
            const int64_t t = GetTimeMicros();
            phaseMicros[ph].fetch_add(t - tSub, std::memory_order_relaxed);
            tSub = t;
        };
        const size_t tcap = pf->tcap, scap = pf->scap;
        const std::vector<int32_t>& tslot = pf->tslot; // block-local txid -> index
        auto findTx = [&](const uint256& txid) -> int {
            size_t h = ReadLE64(txid.begin()) & (tcap - 1);
            while (tslot[h] >= 0) {
                if (block.vtx[tslot[h]]->GetHash() == txid) return tslot[h];
                h = (h + 1) & (tcap - 1);
            }
            return -1;
        };
        const std::vector<size_t>& firstOutput = pf->firstOutput;
        std::atomic<uint8_t>* outSpent = pf->outSpent.get();
        // concurrent set of spent outpoints (input index + 1 per slot): a second spend of one
        // outpoint within the block is found by whichever insert comes second
        std::atomic<uint32_t>* spentSet = pf->spentSet.get();
        const std::vector<size_t>& inputTx = pf->inputTx;
        auto prevoutOf = [&](size_t k) -> const COutPoint& {
            return block.vtx[inputTx[k]]->vin[k - firstInput[inputTx[k]]].prevout;
        };
        auto insertSpent = [&](const COutPoint& op, size_t k) -> bool {
            size_t h = (ReadLE64(op.hash.begin()) ^ ((uint64_t)op.n * 0x9E3779B97F4A7C15ULL)) & (scap - 1);
            for (;;) {
                uint32_t cur = spentSet[h].load(std::memory_order_acquire);
                if (cur == 0) {
                    if (spentSet[h].compare_exchange_strong(cur, (uint32_t)(k + 1), std::memory_order_acq_rel)) return true;
                }
                if (cur != 0 && prevoutOf(cur - 1) == op) return false; // spent twice in this block
                if (cur != 0) h = (h + 1) & (scap - 1);
            }
        };
        enum : uint8_t { SRC_PREFETCH = 0, SRC_VIEW = 1, SRC_BLOCK = 2 };
        std::vector<const Coin*> coinOf(maxJobs, nullptr);
        const size_t TCHUNK = 32; // transactions per task of the parallel pass
        made.resize((ntx + TCHUNK - 1) / TCHUNK);
        std::vector<uint8_t> src(maxJobs, SRC_PREFETCH);
        std::vector<uint64_t> txSigOps(ntx, 0);
        std::vector<Amount> txFee(ntx, 0);
        std::atomic<bool> bad{false};
        txSigOps[0] = legacySigOps[0];
        sub(PH_FU_SETUP);
        pool->ParallelFor(
            (ntx + TCHUNK - 1) / TCHUNK,
            [&](size_t chunk) {
                std::vector<int> heights;
                for (size_t i = std::max<size_t>(1, chunk * TCHUNK); i < std::min(ntx, (chunk + 1) * TCHUNK); i++) {
                    if (bad.load(std::memory_order_relaxed)) return;
                    const CTransaction& tx = *block.vtx[i];
                    bool ok = true;
                    for (size_t j = 0; j < tx.vin.size() && ok; j++) {
                        const size_t k = firstInput[i] + j;
                        const COutPoint& op = tx.vin[j].prevout;
                        const Coin* c = view.FindInCache(op);
                        const int t = findTx(op.hash);
                        if (c) {
                            if (t >= 0) ok = false; // the view already holds an output of this block: serial pass
                            src[k] = SRC_VIEW;
                        } else if (t >= 0) {
                            const CTransaction& ptx = *block.vtx[t];
                            if (t >= (int)i || op.n >= ptx.vout.size() || ptx.vout[op.n].scriptPubKey.IsUnspendable()) {
                                ok = false;
                            } else {
                                made[chunk].emplace_back(ptx.vout[op.n], pindex->nHeight, t == 0);
                                c = &made[chunk].back();
                                src[k] = SRC_BLOCK;
                                outSpent[firstOutput[t] + op.n].store(1, std::memory_order_relaxed);
                            }
                        } else if (prefetchedFound[k]) {
                            c = &prefetched[k];
                        }
                        if (!ok || !c || c->IsSpent() || !insertSpent(op, k)) {
                            ok = false;
                            break;
                        }
                        coinOf[k] = c;
                    }
                    if (ok) {
                        heights.resize(tx.vin.size());
                        for (size_t j = 0; j < tx.vin.size(); j++) heights[j] = coinOf[firstInput[i] + j]->GetHeight();
                        ok = SequenceLocks(tx, nLockTimeFlags, &heights, *pindex);
                    }
                    if (ok) {
                        uint64_t so = legacySigOps[i];
                        if (flags & SCRIPT_VERIFY_P2SH)
                            for (size_t j = 0; j < tx.vin.size(); j++) {
                                const CScript& spk = coinOf[firstInput[i] + j]->GetTxOut().scriptPubKey;
                                if (spk.IsPayToScriptHash()) so += spk.GetSigOpCount(tx.vin[j].scriptSig);
                            }
                        txSigOps[i] = so;
                        ok = so <= MAX_TX_SIGOPS_COUNT;
                    }
                    if (ok) {
                        Amount in = 0;
                        for (size_t j = 0; j < tx.vin.size() && ok; j++) {
                            const Coin& c = *coinOf[firstInput[i] + j];
                            if (c.IsCoinBase() && pindex->nHeight - (int)c.GetHeight() < COINBASE_MATURITY) ok = false;
                            in += c.GetTxOut().nValue;
                            if (!MoneyRange(c.GetTxOut().nValue) || !MoneyRange(in)) ok = false;
                        }
                        const Amount out = tx.GetValueOut();
                        if (!ok || in < out || !MoneyRange(in - out)) ok = false;
                        else txFee[i] = in - out;
                    }
                    if (!ok) bad.store(true, std::memory_order_relaxed);
                }
            },
            1);
        uint64_t sigTotal = 0;
        sub(PH_FU_CHECKS);
        for (size_t i = 0; i < ntx && !bad.load(); i++) {
            if (txSigOps[i] > MAX_TX_SIGOPS_COUNT) bad = true; // the coinbase's legacy count
            sigTotal += txSigOps[i];
            if (sigTotal > nMaxSigOpsCount) bad = true;
        }
        // In place on the coins tip (ConnectTip): the view is empty, so every input was fetched
        // and nothing of the block is in the view yet. Not when the coinbase would overwrite a
        // coin (a duplicate coinbase after BIP34; undoing it could not bring that coin back).
        CCoinsViewCache* tip = p.directTip;
        if (!bad.load() && tip && view.GetCacheSize() == 0) {
            const CTransaction& cb = *block.vtx[0];
            for (size_t o = 0; o < cb.vout.size() && tip; o++)
                if (tip->HaveCoin(COutPoint(cb.GetHash(), (uint32_t)o))) tip = nullptr;
        } else {
            tip = nullptr;
        }
        CCoinsViewCache& target = tip ? *tip : view;
        if (!bad.load()) {
            fastDone = true;
            phaseMicros[PH_FASTUTXO].fetch_add(1, std::memory_order_relaxed);
            // Script jobs first, so the scripts run under the rest of the pass: each job reads its
            // spent coin where the checks found it (the prefetched copy, or `made` for an output of
            // this block and for a copy of a coin the view holds, which the updates below change)
            std::vector<uint8_t> needScripts(ntx, 0);
            pool->ParallelFor(
                (ntx + TCHUNK - 1) / TCHUNK,
                [&](size_t chunk) {
                    for (size_t i = std::max<size_t>(1, chunk * TCHUNK); i < std::min(ntx, (chunk + 1) * TCHUNK); i++) {
                        needScripts[i] = fScriptChecks && !(scMayHold && sc.Has(scKeys[i], !fJustCheck));
                        for (size_t k = firstInput[i]; k < firstInput[i + 1]; k++)
                            if (src[k] == SRC_VIEW) {
                                made[chunk].push_back(*coinOf[k]);
                                coinOf[k] = &made[chunk].back();
                            }
                    }
                },
                1);
            std::vector<size_t> jobOff(ntx + 1, 0);
            for (size_t i = 0; i < ntx; i++) jobOff[i + 1] = jobOff[i] + (needScripts[i] ? block.vtx[i]->vin.size() : 0);
            pool->ParallelFor(
                ntx,
                [&](size_t i) {
                    if (!needScripts[i]) return;
                    const CTransaction& tx = *block.vtx[i];
                    for (size_t j = 0; j < tx.vin.size(); j++) {
                        const CTxOut& out = coinOf[firstInput[i] + j]->GetTxOut();
                        jobs[jobOff[i] + j] = ScriptJob{&tx, (unsigned)j, &out.scriptPubKey, out.nValue, txdatas[i].get()};
                    }
                },
                64);
            nProduced = jobOff[ntx];
            if (queued && nProduced > 0) {
                scriptQueue->Publish(nProduced);
                nPublished = nProduced;
            }
            // A check-only connect (TestBlockValidity) discards its view and writes no undo record:
            // the verdict needs neither, so the records and the view updates are skipped (the
            // checks above already resolved every input, spends inside the block included).
            // Otherwise: undo records (copies of the spent coins: the scripts read the originals)
            std::vector<Coin> newCoins; // the block's outputs that stay unspent, built here
            std::vector<uint8_t> inShard, outShard; // CCoinsMap::ShardOf of each input / output
            if (!fJustCheck) {
                blockundo.vtxundo.resize(ntx - 1);
                newCoins.resize(nOutputs);
                inShard.resize(maxJobs);
                outShard.resize(nOutputs);
                pool->ParallelFor(
                    (ntx + TCHUNK - 1) / TCHUNK,
                    [&](size_t chunk) {
                        for (size_t i = std::max<size_t>(1, chunk * TCHUNK); i < std::min(ntx, (chunk + 1) * TCHUNK); i++) {
                            const CTransaction& tx = *block.vtx[i];
                            CTxUndo& undo = blockundo.vtxundo[i - 1];
                            undo.vprevout.resize(tx.vin.size());
                            for (size_t j = 0; j < tx.vin.size(); j++) undo.vprevout[j] = *coinOf[firstInput[i] + j];
                        }
                        for (size_t i = chunk * TCHUNK; i < std::min(ntx, (chunk + 1) * TCHUNK); i++) {
                            const CTransaction& tx = *block.vtx[i];
                            for (size_t j = 0; i > 0 && j < tx.vin.size(); j++)
                                inShard[firstInput[i] + j] = (uint8_t)CCoinsMap::ShardOf(tx.vin[j].prevout);
                            for (size_t o = 0; o < tx.vout.size(); o++)
                                outShard[firstOutput[i] + o] = (uint8_t)CCoinsMap::ShardOf(COutPoint(tx.GetHash(), (uint32_t)o));
                            for (size_t o = 0; o < tx.vout.size(); o++)
                                if (!outSpent[firstOutput[i] + o].load(std::memory_order_relaxed) &&
                                    !tx.vout[o].scriptPubKey.IsUnspendable())
                                    newCoins[firstOutput[i] + o] = Coin(tx.vout[o], pindex->nHeight, i == 0);
                        }
                    },
                    1);
            }
            sub(PH_FU_UNDO);
            for (size_t i = 0; i < ntx; i++) {
                nInputs += (int)block.vtx[i]->vin.size();
                nFees += txFee[i];
                vPos.push_back(std::make_pair(block.vtx[i]->GetHash(), pos));
                pos.nTxOffset += txSizes[i];
            }
            nSigOpsCount = sigTotal;
            // The view updates (or the tip's), one coins-map shard per task (CCoinsMap): spends of
            // fetched coins and of the view's own coins, then the block's outputs that stay
            // unspent. The scripts published above run meanwhile; nothing they read is in the view.
            std::string applyError;
            std::mutex applyMu;
            if (!fJustCheck) {
                if (!tip) view.Reserve(view.GetCacheSize() + maxJobs + nOutputs);
                p.tipApplied = tip != nullptr;
                target.ForEachShard(
                    [&](unsigned sh) {
                        try {
                            for (size_t k = 0; k < maxJobs; k++) {
                                if (inShard[k] != sh) continue;
                                const COutPoint& op = prevoutOf(k);
                                if (src[k] == SRC_BLOCK) continue; // created and spent inside the block: no entry
                                if (tip) tip->SpendPeeked(op);
                                else if (src[k] == SRC_PREFETCH) view.SpendFetchedMoved(op);
                                else if (src[k] == SRC_VIEW && !view.SpendCoin(op)) throw std::runtime_error("view spend failed");
                            }
                            for (size_t i = 0; i < ntx; i++) {
                                const CTransaction& tx = *block.vtx[i];
                                for (size_t o = 0; o < tx.vout.size(); o++) {
                                    const size_t q = firstOutput[i] + o;
                                    if (outShard[q] == sh && !newCoins[q].IsSpent())
                                        target.AddCoin(COutPoint(tx.GetHash(), (uint32_t)o), std::move(newCoins[q]), i == 0);
                                }
                            }
                        } catch (const std::exception& e) {
                            std::lock_guard<std::mutex> l(applyMu);
                            applyError = e.what();
                        }
                    },
                    pool.get());
            }
            sub(PH_FU_APPLY);
            if (!applyError.empty()) return state.Error("ConnectBlock: " + applyError);
        }
    }
    if (!fastDone) {
        // the view gains about one entry per input and output: size its table once
        view.Reserve(view.GetCacheSize() + maxJobs + nOutputs);
        // The serial UTXO pass. Each input's coin is taken from the view (or the prefetch) once; the
        // checks below used to go back to the view for it six times (HaveInputs, the height list,
        // the P2SH sigop count, GetValueIn, CheckTxInputs, SpendCoin). The references stay valid
        // while the view grows.
        std::vector<const Coin*> coins;
        std::vector<uint8_t> fromPrefetch;
        for (size_t i = 0; i < ntx; i++) {
            const CTransaction& tx = *block.vtx[i];
            nInputs += (int)tx.vin.size();
            if (!tx.IsCoinBase()) {
                coins.resize(tx.vin.size());
                fromPrefetch.resize(tx.vin.size());
                for (size_t j = 0; j < tx.vin.size(); j++) {
                    // the view's own entry (a coin created or spent earlier in the block) wins
                    const size_t k = firstInput[i] + j;
                    const Coin* c = view.FindInCache(tx.vin[j].prevout);
                    fromPrefetch[j] = c == nullptr;
                    if (!c && prefetchedFound[k]) c = &prefetched[k];
                    if (!c || c->IsSpent())
                        return state.DoS(100, error("ConnectBlock(): inputs missing/spent"), REJECT_INVALID,
                                         "bad-txns-inputs-missingorspent");
                    coins[j] = c;
                }
                prevheights.resize(tx.vin.size());
                for (size_t j = 0; j < tx.vin.size(); j++) prevheights[j] = coins[j]->GetHeight();
                if (!SequenceLocks(tx, nLockTimeFlags, &prevheights, *pindex))
                    return state.DoS(100, error("%s: contains a non-BIP68-final transaction", __func__), REJECT_INVALID,
                                     "bad-txns-nonfinal");
            }
            // GetTransactionSigOpCount over the looked-up coins
            uint64_t txSigOps = legacySigOps[i];
            if (!tx.IsCoinBase() && (flags & SCRIPT_VERIFY_P2SH))
                for (size_t j = 0; j < tx.vin.size(); j++) {
                    const CScript& spk = coins[j]->GetTxOut().scriptPubKey;
                    if (spk.IsPayToScriptHash()) txSigOps += spk.GetSigOpCount(tx.vin[j].scriptSig);
                }
            if (txSigOps > MAX_TX_SIGOPS_COUNT) return state.DoS(100, false, REJECT_INVALID, "bad-txn-sigops");
            nSigOpsCount += txSigOps;
            if (nSigOpsCount > nMaxSigOpsCount)
                return state.DoS(100, error("ConnectBlock(): too many sigops"), REJECT_INVALID, "bad-blk-sigops");
            if (!tx.IsCoinBase()) {
                // Consensus::CheckTxInputs over the looked-up coins; on any failure the original runs
                // for the exact reject reason
                Amount in = 0;
                bool ok = true;
                for (size_t j = 0; j < tx.vin.size() && ok; j++) {
                    const Coin& c = *coins[j];
                    if (c.IsCoinBase() && pindex->nHeight - (int)c.GetHeight() < COINBASE_MATURITY) ok = false;
                    in += c.GetTxOut().nValue;
                    if (!MoneyRange(c.GetTxOut().nValue) || !MoneyRange(in)) ok = false;
                }
                const Amount out = tx.GetValueOut();
                if (!ok || in < out || !MoneyRange(in - out)) {
                    if (!Consensus::CheckTxInputs(tx, state, view, pindex->nHeight))
                        return error("ConnectBlock(): CheckTxInputs on %s failed with %s", tx.GetHash().ToString().c_str(),
                                     FormatStateMessage(state).c_str());
                    return state.Error("ConnectBlock: input checks disagree");
                }
                nFees += in - out;
            }
            CTxUndo undoDummy;
            if (i > 0) blockundo.vtxundo.push_back(CTxUndo());
            CTxUndo& undo = i == 0 ? undoDummy : blockundo.vtxundo.back();
            if (!tx.IsCoinBase()) {
                undo.vprevout.reserve(tx.vin.size());
                for (size_t j = 0; j < tx.vin.size(); j++) {
                    undo.vprevout.emplace_back();
                    if (fromPrefetch[j])
                        view.SpendFetched(tx.vin[j].prevout, std::move(prefetched[firstInput[i] + j]), &undo.vprevout.back());
                    else if (!view.SpendCoin(tx.vin[j].prevout, &undo.vprevout.back()))
                        return state.Error("ConnectBlock: spend failed");
                }
                // transactions fully validated under these flags in the mempool skip re-execution; the
                // jobs read the spent coins from the undo record (reserved up front: the addresses are
                // stable for the whole block) instead of copying each script
                if (fScriptChecks && !(scMayHold && sc.Has(scKeys[i], !fJustCheck))) {
                    for (size_t j = 0; j < tx.vin.size(); j++) {
                        const CTxOut& out = undo.vprevout[j].GetTxOut();
                        jobs[nProduced + j] = ScriptJob{&tx, (unsigned)j, &out.scriptPubKey, out.nValue, txdatas[i].get()};
                    }
                    nProduced += tx.vin.size();
                    // publish in groups: each publish takes the queue lock and may wake a worker
                    if (nProduced - nPublished >= 512) {
                        scriptQueue->Publish(nProduced);
                        nPublished = nProduced;
                    }
                }
            }
            AddCoins(view, tx, pindex->nHeight);
            vPos.push_back(std::make_pair(tx.GetHash(), pos));
            pos.nTxOffset += txSizes[i];
        }
    }
    const int64_t nTime2 = GetTimeMicros();
    phase(PH_UTXO);

    const Amount blockReward = nFees + GetBlockSubsidy(pindex->nHeight, cp);
    if (block.vtx[0]->GetValueOut() > blockReward)
        return state.DoS(100,
                         error("ConnectBlock(): coinbase pays too much (actual=%lld vs limit=%lld)",
                               (long long)block.vtx[0]->GetValueOut(), (long long)blockReward),
                         REJECT_INVALID, "bad-cb-amount");

    // ---- remaining scripts, then one ECDSA batch (GPU when large enough)
    scriptQueue->Publish(nProduced);
    scriptQueue->Complete();
    phase(PH_SCRIPTS);
    const size_t nJobs = nProduced;
    p.nJobs = nJobs;
    p.postfork = postfork;
    p.nInputs = nInputs;
    p.nTime2 = nTime2;
    if (nJobs > 0) {
        bool ok = !anyFail.load();
        if (ok) {
            // the batch reads the checks where the jobs left them: a pointer per check
            std::vector<size_t> off(nJobs + 1, 0);
            for (size_t k = 0; k < nJobs; k++) off[k + 1] = off[k] + sinks[k].size();
            std::vector<const DeferredSigCheck*> all(off[nJobs]);
            std::vector<DeferredMultisig> groups;
            for (size_t k = 0; k < nJobs; k++)
                for (DeferredMultisig g : groupSinks[k]) { // rebase onto the flat numbering
                    g.first += (uint32_t)off[k];
                    groups.push_back(g);
                }
            pool->ParallelFor(
                nJobs,
                [&](size_t k) {
                    for (size_t j = 0; j < sinks[k].size(); j++) all[off[k] + j] = &sinks[k][j];
                },
                512);
            phase(PH_COLLECT);
            {
                // While the GPU checks the signatures the CPU is idle: the undo record is
                // serialised and checksummed meanwhile (written once the verdict is in)
                if (!fJustCheck && pindex->GetUndoPos().IsNull() && ntx >= 1024 && GpuBatchesExpected(opts.useGpu)) {
                    const CBlockUndo* u = &blockundo;
                    const uint256 prevHash = pindex->pprev->GetBlockHash();
                    WorkerPool* wp = pool.get(); // idle meanwhile unless the batch probes the cache
                    p.undoSer = std::async(std::launch::async, [u, prevHash, wp]() {
                        std::vector<unsigned char> ser = SerializeBlockUndo(*u, wp);
                        const uint256 sum = UndoChecksum(ser, prevHash);
                        return std::make_pair(std::move(ser), sum);
                    });
                }
                // the scripts' session is closed: the next block's read-only pass may use the queue
                if (!fJustCheck && opts.connectLookahead && p.tipApplied && ntx >= 1024 && GpuBatchesExpected(opts.useGpu)) {
                    completeOnExit.armed = false;
                    StartLookahead(pindex);
                }
                ok = BatchVerifySignatures(all, groups, pool.get(), opts.useGpu, false, !fJustCheck);
                phase(PH_BATCH);
            }
        }
        p.sigsOk = ok;
    }
    if (!fJustCheck) view.SetBestBlock(pindex->GetBlockHash());
    // a big block leaves ~100k heap objects in these: freed on the reaper thread
    if (ntx >= 1024) {
        Reaper::Get().Drop(std::move(sinks));
        Reaper::Get().Drop(std::move(groupSinks));
        Reaper::Get().Drop(std::move(txdatas));
        Reaper::Get().Drop(std::move(prefetched));
    }
    return true;
}

// Phase 2: wait for the signature verdict, then record the block as script-valid (undo data,
// index status, tx index). On failure nothing of the block has been committed.
bool Chainstate::ConnectBlockFinish(PendingConnect& p, CValidationState& state, bool fJustCheck) {
    if (p.genesis) return true;
    CBlockIndex* pindex = p.pindex;
    const CBlockUndo& blockundo = p.blockundo;
    const bool ok = p.sigsOk;
    // Before the fork script failures do not invalidate blocks (reference validation.cpp:2121-2126:
    // control.Wait() is ignored below BCPHeight; the checks always go through the queue control,
    // :2010-2011 and :2080-2087, whatever -par says, so this holds for every thread count).
    if (p.nJobs > 0 && !ok && p.postfork)
        return state.DoS(100, false, REJECT_INVALID, "blk-bad-inputs", false, "parallel script check failed");
    const int64_t nTime4 = GetTimeMicros();
    LogPrint(BCLog::BENCH, "    - Connect %d inputs (%zu script jobs): %.2fms, verify %.2fms\n", p.nInputs, p.nJobs,
             0.001 * (p.nTime2 - p.nTimeStart), 0.001 * (nTime4 - p.nTime2));
    if (fJustCheck) return true;

    if (pindex->GetUndoPos().IsNull() || !pindex->IsValid(BLOCK_VALID_SCRIPTS)) {
        if (pindex->GetUndoPos().IsNull()) {
            const int64_t tu = GetTimeMicros();
            CDiskBlockPos upos;
            std::vector<unsigned char> ser;
            uint256 sum;
            const bool early = p.undoSer.valid();
            if (early) std::tie(ser, sum) = p.undoSer.get();
            else ser = SerializeBlockUndo(blockundo, pool.get());
            if (!FindUndoPos(state, pindex->nFile, upos, (unsigned)ser.size() + 40))
                return error("ConnectBlock(): FindUndoPos failed");
            if (!UndoWriteToDisk(ser, upos, pindex->pprev->GetBlockHash(), params.DiskMagic(), early ? &sum : nullptr))
                return state.Error("Failed to write undo data");
            pindex->nUndoPos = upos.nPos;
            pindex->nStatus |= BLOCK_HAVE_UNDO;
            phaseMicros[PH_UNDO].fetch_add(GetTimeMicros() - tu, std::memory_order_relaxed);
        }
        pindex->RaiseValidity(BLOCK_VALID_SCRIPTS);
        setDirtyBlockIndex.insert(pindex);
    }
    if (opts.txindex && !pblocktree->WriteTxIndex(p.vPos)) return state.Error("Failed to write transaction index");
    nLastConnectMicros = GetTimeMicros() - p.nTimeStart;
    return true;
}

static DisconnectResult UndoCoinSpend(const Coin& undo, CCoinsViewCache& view, const COutPoint& out) {
    bool fClean = true;
    if (view.HaveCoin(out)) fClean = false; // overwriting transaction output
    if (undo.GetHeight() == 0) {
        // pre-0.15 undo records lacked height/coinbase: recover them from another output of the tx
        const Coin& alternate = AccessByTxid(view, out.hash);
        if (alternate.IsSpent()) return DISCONNECT_FAILED;
        Coin c = undo;
        c.nHeight = alternate.nHeight;
        c.fCoinBase = alternate.fCoinBase;
        view.AddCoin(out, std::move(c), !fClean);
        return fClean ? DISCONNECT_OK : DISCONNECT_UNCLEAN;
    }
    Coin c = undo;
    view.AddCoin(out, std::move(c), !fClean);
    return fClean ? DISCONNECT_OK : DISCONNECT_UNCLEAN;
}

DisconnectResult ApplyBlockUndo(const CBlockUndo& blockUndo, const CBlock& block, const CBlockIndex* pindex,
                                CCoinsViewCache& view) {
    if (blockUndo.vtxundo.size() + 1 != block.vtx.size()) {
        error("DisconnectBlock(): block and undo data inconsistent");
        return DISCONNECT_FAILED;
    }
    bool fClean = true;
    for (int i = (int)block.vtx.size() - 1; i >= 0; i--) {
        const CTransaction& tx = *block.vtx[i];
        const uint256& txid = tx.GetHash();
        // outputs must be unspent; remove them
        for (size_t o = 0; o < tx.vout.size(); o++) {
            if (tx.vout[o].scriptPubKey.IsUnspendable()) continue;
            COutPoint out(txid, (uint32_t)o);
            Coin coin;
            const bool is_spent = view.SpendCoin(out, &coin);
            if (!is_spent || tx.vout[o] != coin.GetTxOut() || (uint32_t)pindex->nHeight != coin.GetHeight() ||
                tx.IsCoinBase() != coin.IsCoinBase())
                fClean = false;
        }
        if (i > 0) {
            const CTxUndo& txundo = blockUndo.vtxundo[i - 1];
            if (txundo.vprevout.size() != tx.vin.size()) {
                error("DisconnectBlock(): transaction and undo data inconsistent");
                return DISCONNECT_FAILED;
            }
            for (size_t j = tx.vin.size(); j-- > 0;) {
                const DisconnectResult res = UndoCoinSpend(txundo.vprevout[j], view, tx.vin[j].prevout);
                if (res == DISCONNECT_FAILED) return DISCONNECT_FAILED;
                fClean = fClean && res != DISCONNECT_UNCLEAN;
            }
        }
    }
    view.SetBestBlock(block.hashPrevBlock);
    return fClean ? DISCONNECT_OK : DISCONNECT_UNCLEAN;
}

void UpdateCoins(const CTransaction& tx, CCoinsViewCache& view, CTxUndo& txundo, int nHeight) {
    if (!tx.IsCoinBase()) {
        txundo.vprevout.reserve(tx.vin.size());
        for (const CTxIn& in : tx.vin) {
            txundo.vprevout.emplace_back();
            const bool spent = view.SpendCoin(in.prevout, &txundo.vprevout.back());
            assert(spent);
        }
    }
    AddCoins(view, tx, nHeight);
}

void UpdateCoins(const CTransaction& tx, CCoinsViewCache& view, int nHeight) {
    CTxUndo txundo;
    UpdateCoins(tx, view, txundo, nHeight);
}

DisconnectResult Chainstate::DisconnectBlock(const CBlock& block, const CBlockIndex* pindex, CCoinsViewCache& view) {
    CBlockUndo blockUndo;
    CDiskBlockPos pos = pindex->GetUndoPos();
    if (pos.IsNull()) {
        error("DisconnectBlock(): no undo data available");
        return DISCONNECT_FAILED;
    }
    if (!UndoReadFromDisk(blockUndo, pos, pindex->pprev->GetBlockHash())) {
        error("DisconnectBlock(): failure reading undo data");
        return DISCONNECT_FAILED;
    }
    return ApplyBlockUndo(blockUndo, block, pindex, view);
}

// ------------------------------------------------------------------ flushing
uint64_t Chainstate::CalculateCurrentUsage() const {
    uint64_t r = 0;
    for (const CBlockFileInfo& f : vinfoBlockFile) r += f.nSize + f.nUndoSize;
    return r;
}

bool Chainstate::FlushStateToDisk(CValidationState& state, FlushStateMode mode, int nManualPruneHeight) {
    std::lock_guard<CCriticalSection> l(cs_main);
    const int64_t nMempoolUsage = mempool ? (int64_t)mempool->DynamicMemoryUsage() : 0;
    std::set<int> setFilesToPrune;
    bool fFlushForPrune = false;
    try {
        if (PruneMode() && (fCheckForPruning || nManualPruneHeight > 0) && !fReindex) {
            if (nManualPruneHeight > 0) FindFilesToPruneManual(setFilesToPrune, nManualPruneHeight);
            else FindFilesToPrune(setFilesToPrune, params.PruneAfterHeight());
            fCheckForPruning = false;
            if (!setFilesToPrune.empty()) {
                fFlushForPrune = true;
                if (!fHavePruned) {
                    pblocktree->WriteFlag("prunedblockfiles", true);
                    fHavePruned = true;
                }
            }
        }
        const int64_t nNow = GetTimeMicros();
        if (nLastWrite == 0) nLastWrite = nNow;
        if (nLastFlush == 0) nLastFlush = nNow;
        if (nLastSetChain == 0) nLastSetChain = nNow;
        const int64_t nMempoolSizeMax = gArgs.GetArg("-maxmempool", (int64_t)DEFAULT_MAX_MEMPOOL_SIZE) * 1000000;
        const int64_t cacheSize = (int64_t)pcoinsTip->DynamicMemoryUsage();
        const int64_t nTotalSpace = (int64_t)opts.coinsCacheBytes + std::max<int64_t>(nMempoolSizeMax - nMempoolUsage, 0);
        const bool fCacheLarge = mode == FLUSH_STATE_PERIODIC &&
                                 cacheSize > std::max((9 * nTotalSpace) / 10, nTotalSpace - (int64_t)(10u << 20));
        const bool fCacheCritical = mode == FLUSH_STATE_IF_NEEDED && cacheSize > nTotalSpace;
        const bool fPeriodicWrite = mode == FLUSH_STATE_PERIODIC && nNow > nLastWrite + (int64_t)DATABASE_WRITE_INTERVAL * 1000000;
        const bool fPeriodicFlush = mode == FLUSH_STATE_PERIODIC && nNow > nLastFlush + (int64_t)DATABASE_FLUSH_INTERVAL * 1000000;
        const bool fDoFullFlush = (mode == FLUSH_STATE_ALWAYS) || fCacheLarge || fCacheCritical || fPeriodicFlush || fFlushForPrune;
        if (fDoFullFlush || fPeriodicWrite) {
            FlushBlockFile();
            std::vector<std::pair<int, const CBlockFileInfo*>> vFiles;
            for (int f : setDirtyFileInfo) vFiles.push_back(std::make_pair(f, &vinfoBlockFile[f]));
            setDirtyFileInfo.clear();
            std::vector<const CBlockIndex*> vBlocks(setDirtyBlockIndex.begin(), setDirtyBlockIndex.end());
            setDirtyBlockIndex.clear();
            if (!pblocktree->WriteBatchSync(vFiles, nLastBlockFile, vBlocks))
                return state.Error("Failed to write to block index database");
            if (fFlushForPrune) UnlinkPrunedFiles(setFilesToPrune);
            nLastWrite = nNow;
        }
        if (fDoFullFlush) {
            if (!pcoinsTip->Flush()) return state.Error("Failed to write to coin database");
            nLastFlush = nNow;
        }
        if (fDoFullFlush || ((mode == FLUSH_STATE_ALWAYS || mode == FLUSH_STATE_PERIODIC) &&
                             nNow > nLastSetChain + (int64_t)DATABASE_WRITE_INTERVAL * 1000000)) {
            if (chainActive.Tip()) GetMainSignals().SetBestChain(chainActive.GetLocator());
            nLastSetChain = nNow;
        }
    } catch (const std::runtime_error& e) {
        return state.Error(std::string("System error while flushing: ") + e.what());
    }
    return true;
}

void Chainstate::FlushStateToDisk() {
    CValidationState state;
    FlushStateToDisk(state, FLUSH_STATE_ALWAYS);
}

// ------------------------------------------------------------------ tip management
namespace {
// Reference validation.cpp:1770 WarningBitsConditionChecker: a version bit this node does not
// set itself that a BIP9 window's threshold of blocks signals (begin 0, never times out).
class WarningBitsConditionChecker : public AbstractThresholdConditionChecker {
    int bit;
    VersionBitsCache& vbcache;

public:
    WarningBitsConditionChecker(int bitIn, VersionBitsCache& c) : bit(bitIn), vbcache(c) {}
    int64_t BeginTime(const Consensus::Params&) const override { return 0; }
    int64_t EndTime(const Consensus::Params&) const override { return std::numeric_limits<int64_t>::max(); }
    int Period(const Consensus::Params& p) const override { return p.nMinerConfirmationWindow; }
    int Threshold(const Consensus::Params& p) const override { return p.nRuleChangeActivationThreshold; }
    bool Condition(const CBlockIndex* pindex, const Consensus::Params& p) const override {
        return (pindex->nVersion & VERSIONBITS_TOP_MASK) == VERSIONBITS_TOP_BITS && ((pindex->nVersion >> bit) & 1) != 0 &&
               ((bcp::ComputeBlockVersion(pindex->pprev, p, vbcache) >> bit) & 1) == 0;
    }
};
} // namespace

// Reference validation.cpp:2348 UpdateTip: besides moving the tip, warn (and -alertnotify once)
// about unknown rules: a versionbit that locked in / activated without this node knowing it, or
// more than half of the last 100 blocks carrying bits this node would not set.
void Chainstate::UpdateTip(CBlockIndex* pindexNew) {
    chainActive.SetTip(pindexNew);
    if (mempool) mempool->AddTransactionsUpdated(1);
    cvBlockChange.notify_all();
    std::string strWarning;
    std::vector<std::string> warningMessages;
    if (!IsInitialBlockDownload()) {
        const CBlockIndex* pindex = chainActive.Tip();
        for (int bit = 0; bit < VERSIONBITS_NUM_BITS; bit++) {
            WarningBitsConditionChecker checker(bit, versionbitscache);
            const ThresholdState state = checker.GetStateFor(pindex, params.GetConsensus(), warningcache[bit]);
            if (state == THRESHOLD_ACTIVE) {
                strWarning = strprintf("Warning: unknown new rules activated (versionbit %i)", bit);
                if (!fUnknownRulesWarned) {
                    AlertNotify(strWarning);
                    fUnknownRulesWarned = true;
                }
            } else if (state == THRESHOLD_LOCKED_IN) {
                warningMessages.push_back(strprintf("unknown new rules are about to activate (versionbit %i)", bit));
            }
        }
        int nUpgraded = 0;
        for (int i = 0; i < 100 && pindex != nullptr; i++) {
            const int32_t nExpectedVersion = bcp::ComputeBlockVersion(pindex->pprev, params.GetConsensus(), versionbitscache);
            if (pindex->nVersion > VERSIONBITS_LAST_OLD_BLOCK_VERSION && (pindex->nVersion & ~nExpectedVersion) != 0)
                ++nUpgraded;
            pindex = pindex->pprev;
        }
        if (nUpgraded > 0) warningMessages.push_back(strprintf("%d of last 100 blocks have unexpected version", nUpgraded));
        if (nUpgraded > 100 / 2) {
            strWarning = "Warning: Unknown block versions being mined! It's possible unknown rules are in effect";
            if (!fUnknownRulesWarned) {
                AlertNotify(strWarning);
                fUnknownRulesWarned = true;
            }
        }
    }
    if (!strWarning.empty()) bcp::SetMiscWarning(strWarning);
    LogPrintf("UpdateTip: new best=%s height=%d version=0x%08x log2_work=%.8g tx=%lu date='%lld' cache=%.1fMiB(%utxo)\n",
              chainActive.Tip()->GetBlockHash().ToString().c_str(), chainActive.Height(), chainActive.Tip()->nVersion,
              std::log(chainActive.Tip()->nChainWork.getdouble()) / std::log(2.0),
              (unsigned long)chainActive.Tip()->nChainTx, (long long)chainActive.Tip()->GetBlockTime(),
              pcoinsTip->DynamicMemoryUsage() * (1.0 / (1 << 20)), pcoinsTip->GetCacheSize());
    if (!warningMessages.empty()) {
        std::string joined;
        for (const auto& w : warningMessages) joined += (joined.empty() ? "" : ", ") + w;
        LogPrintf("UpdateTip: warning='%s'\n", joined.c_str());
    }
}

bool Chainstate::ReadBlock(CBlock& block, const CBlockIndex* pindex, bool checkPow) const {
    return ReadBlockFromDisk(block, pindex, params, checkPow);
}

bool Chainstate::DisconnectTip(CValidationState& state, bool fBare) {
    JoinLookahead();
    lookahead.reset(); // it read the tip this disconnect changes
    CBlockIndex* pindexDelete = chainActive.Tip();
    auto pblock = std::make_shared<CBlock>();
    if (!ReadBlockFromDisk(*pblock, pindexDelete, params)) return state.Error("Failed to read block");
    {
        CCoinsViewCache view(pcoinsTip.get());
        if (DisconnectBlock(*pblock, pindexDelete, view) != DISCONNECT_OK)
            return error("DisconnectTip(): DisconnectBlock %s failed", pindexDelete->GetBlockHash().ToString().c_str());
        view.Flush();
    }
    if (!FlushStateToDisk(state, FLUSH_STATE_IF_NEEDED)) return false;
    UpdateTip(pindexDelete->pprev);
    if (!fBare && mempool) UpdateMempoolForReorg(pblock->vtx, true);
    GetMainSignals().BlockDisconnected(pblock);
    return true;
}

// -debug=bench accumulators of ConnectTip (reference src/validation.cpp:1690-1700 nTimeCheck,
// nTimeForks, nTimeConnect, nTimeVerify, nTimeIndex, nTimeCallbacks, nTimeTotal and
// :2200-2290 ConnectTip's per-step lines): each line shows this block's time and the running
// total since startup. The connect split is the MI355X pipeline's own phases.
namespace {
struct BenchTotals {
    std::atomic<int64_t> read{0}, connect{0}, flush{0}, chainstate{0}, post{0}, total{0};
    std::atomic<int64_t> phase[Chainstate::PH_COUNT] = {};
    std::atomic<int64_t> blocks{0};
};
BenchTotals& Bench() {
    static BenchTotals t;
    return t;
}
// the timed phases (PH_BLOCKS and PH_FASTUTXO are counters)
const char* const kPhaseNames[Chainstate::PH_BLOCKS] = {"Sanity checks", "Prefetch + precompute", "UTXO pass",
                                                       "Script jobs wait", "Collect checks", "Signature batch"};
void BenchLine(const char* indent, const char* what, int64_t micros, std::atomic<int64_t>& acc) {
    const int64_t tot = (acc += micros);
    LogPrint(BCLog::BENCH, "%s- %s: %.2fms [%.2fs]\n", indent, what, 0.001 * micros, 1e-6 * tot);
}
} // namespace

bool Chainstate::ConnectTip(CValidationState& state, CBlockIndex* pindexNew, const std::shared_ptr<const CBlock>& pblock,
                            ConnectTrace& trace) {
    const bool bench = LogAcceptCategory(BCLog::BENCH);
    const int64_t nTime1 = GetTimeMicros();
    int64_t ph0[PH_COUNT];
    if (bench)
        for (int k = 0; k < PH_COUNT; k++) ph0[k] = ConnectPhaseMicros((ConnectPhase)k);
    std::shared_ptr<const CBlock> pthisBlock = TakeRecentBlock(pindexNew->GetBlockHash());
    if (pblock) {
        pthisBlock = pblock;
    } else if (pthisBlock) {
        recentHits.fetch_add(1, std::memory_order_relaxed);
    } else {
        recentMisses.fetch_add(1, std::memory_order_relaxed);
        auto pblockNew = std::make_shared<CBlock>();
        if (!ReadBlockFromDisk(*pblockNew, pindexNew, params, true, pool.get())) return state.Error("Failed to read block");
        pthisBlock = pblockNew;
    }
    trace.blocksConnected.emplace_back(pindexNew, pthisBlock);
    const CBlock& blockConnecting = *pthisBlock;
    const int64_t nTime2 = GetTimeMicros();
    int64_t nTime3, nTime4;
    {
        // a block that takes the parallel UTXO pass updates the tip in place (undone on failure);
        // the view then only carries the new best block
        CCoinsViewCache view(pcoinsTip.get());
        const bool rv = ConnectBlock(blockConnecting, state, pindexNew, view, false, opts.connectInPlace ? pcoinsTip.get() : nullptr);
        GetMainSignals().BlockChecked(blockConnecting, state);
        if (!rv) {
            if (state.IsInvalid()) InvalidBlockFound(pindexNew, state);
            return error("ConnectTip(): ConnectBlock %s failed (%s)", pindexNew->GetBlockHash().ToString().c_str(),
                         FormatStateMessage(state).c_str());
        }
        nTime3 = GetTimeMicros();
        view.Flush();
        nTime4 = GetTimeMicros();
    }
    if (!FlushStateToDisk(state, FLUSH_STATE_IF_NEEDED)) return false;
    const int64_t nTime5 = GetTimeMicros();
    if (mempool) mempool->removeForBlock(blockConnecting.vtx, pindexNew->nHeight);
    UpdateTip(pindexNew);
    const int64_t nTime6 = GetTimeMicros();
    phaseMicros[PH_TIP_READ].fetch_add(nTime2 - nTime1, std::memory_order_relaxed);
    phaseMicros[PH_TIP_CONNECT].fetch_add(nTime3 - nTime2, std::memory_order_relaxed);
    phaseMicros[PH_TIP_FLUSH].fetch_add(nTime4 - nTime3, std::memory_order_relaxed);
    phaseMicros[PH_TIP_WRITE].fetch_add(nTime5 - nTime4, std::memory_order_relaxed);
    phaseMicros[PH_TIP_POST].fetch_add(nTime6 - nTime5, std::memory_order_relaxed);
    if (bench) {
        BenchTotals& B = Bench();
        B.blocks++;
        BenchLine("  ", "Load block from disk", nTime2 - nTime1, B.read);
        for (int k = 0; k < PH_BLOCKS; k++)
            BenchLine("      ", kPhaseNames[k], ConnectPhaseMicros((ConnectPhase)k) - ph0[k], B.phase[k]);
        if (ConnectPhaseMicros(PH_FASTUTXO) > ph0[PH_FASTUTXO]) LogPrint(BCLog::BENCH, "      - (parallel UTXO pass)\n");
        BenchLine("    ", "Connect total", nTime3 - nTime2, B.connect);
        BenchLine("  ", "Flush", nTime4 - nTime3, B.flush);
        BenchLine("  ", "Writing chainstate", nTime5 - nTime4, B.chainstate);
        BenchLine("  ", "Connect postprocess", nTime6 - nTime5, B.post);
        BenchLine("", "Connect block", nTime6 - nTime1, B.total);
    }
    return true;
}

CBlockIndex* Chainstate::FindMostWorkChain() {
    while (true) {
        if (setBlockIndexCandidates.empty()) return nullptr;
        CBlockIndex* pindexNew = *setBlockIndexCandidates.rbegin();
        CBlockIndex* pindexTest = pindexNew;
        bool fInvalidAncestor = false;
        while (pindexTest && !chainActive.Contains(pindexTest)) {
            const bool fFailedChain = pindexTest->nStatus & BLOCK_FAILED_MASK;
            const bool fMissingData = !(pindexTest->nStatus & BLOCK_HAVE_DATA);
            if (fFailedChain || fMissingData) {
                if (fFailedChain && (pindexBestInvalid == nullptr || pindexNew->nChainWork > pindexBestInvalid->nChainWork))
                    pindexBestInvalid = pindexNew;
                CBlockIndex* pindexFailed = pindexNew;
                while (pindexTest != pindexFailed) {
                    if (fFailedChain) pindexFailed->nStatus |= BLOCK_FAILED_CHILD;
                    else if (fMissingData) mapBlocksUnlinked.insert(std::make_pair(pindexFailed->pprev, pindexFailed));
                    setBlockIndexCandidates.erase(pindexFailed);
                    pindexFailed = pindexFailed->pprev;
                }
                setBlockIndexCandidates.erase(pindexTest);
                fInvalidAncestor = true;
                break;
            }
            pindexTest = pindexTest->pprev;
        }
        if (!fInvalidAncestor) return pindexNew;
    }
}

void Chainstate::PruneBlockIndexCandidates() {
    auto it = setBlockIndexCandidates.begin();
    while (it != setBlockIndexCandidates.end() && setBlockIndexCandidates.value_comp()(*it, chainActive.Tip()))
        setBlockIndexCandidates.erase(it++);
}

void Chainstate::InvalidChainFound(CBlockIndex* pindexNew) {
    if (!pindexBestInvalid || pindexNew->nChainWork > pindexBestInvalid->nChainWork) pindexBestInvalid = pindexNew;
    LogPrintf("InvalidChainFound: invalid block=%s height=%d\n", pindexNew->GetBlockHash().ToString().c_str(),
              pindexNew->nHeight);
    CheckForkWarningConditions();
}

// Large-fork / invalid-chain warnings (reference validation.cpp:1203-1297): a competing branch
// that forked within the last 72 blocks and carries 7+ blocks' worth of work past the fork
// point, or an invalid chain 6+ blocks' worth ahead of our tip, raises a warning (which also
// turns on RPC safe mode) and fires -alertnotify once.
void Chainstate::CheckForkWarningConditions() {
    const CBlockIndex* tip = chainActive.Tip();
    if (!tip || IsInitialBlockDownload()) return;
    if (pindexBestForkTip && chainActive.Height() - pindexBestForkTip->nHeight >= 72) pindexBestForkTip = nullptr;
    if (pindexBestForkTip ||
        (pindexBestInvalid && pindexBestInvalid->nChainWork > tip->nChainWork + GetBlockProof(*tip) * 6)) {
        if (!bcp::GetLargeWorkForkFound() && pindexBestForkBase) {
            AlertNotify("Warning: Large-work fork detected, forking after block " +
                        pindexBestForkBase->phashBlock->ToString());
        }
        if (pindexBestForkTip && pindexBestForkBase) {
            LogPrintf("CheckForkWarningConditions: Warning: Large valid fork found\n  forking the chain at height %d "
                      "(%s)\n  lasting to height %d (%s).\n",
                      pindexBestForkBase->nHeight, pindexBestForkBase->phashBlock->ToString().c_str(),
                      pindexBestForkTip->nHeight, pindexBestForkTip->phashBlock->ToString().c_str());
            bcp::SetLargeWorkForkFound(true);
        } else {
            LogPrintf("CheckForkWarningConditions: Warning: Found invalid chain at least ~6 blocks longer than our "
                      "best chain.\n");
            bcp::SetLargeWorkInvalidChainFound(true);
        }
    } else {
        bcp::SetLargeWorkForkFound(false);
        bcp::SetLargeWorkInvalidChainFound(false);
    }
}

std::string Chainstate::Warnings() const { return bcp::GetWarnings("statusbar"); }

void Chainstate::CheckForkWarningConditionsOnNewFork(CBlockIndex* pindexNewForkTip) {
    CBlockIndex* pfork = pindexNewForkTip;
    CBlockIndex* plonger = chainActive.Tip();
    while (pfork && pfork != plonger) {
        while (plonger && plonger->nHeight > pfork->nHeight) plonger = plonger->pprev;
        if (pfork == plonger) break;
        pfork = pfork->pprev;
    }
    if (pfork && (!pindexBestForkTip || pindexNewForkTip->nHeight > pindexBestForkTip->nHeight) &&
        pindexNewForkTip->nChainWork - pfork->nChainWork > GetBlockProof(*pfork) * 7 &&
        chainActive.Height() - pindexNewForkTip->nHeight < 72) {
        pindexBestForkTip = pindexNewForkTip;
        pindexBestForkBase = pfork;
    }
    CheckForkWarningConditions();
}

void Chainstate::InvalidBlockFound(CBlockIndex* pindex, const CValidationState& state) {
    if (!state.CorruptionPossible()) {
        pindex->nStatus |= BLOCK_FAILED_VALID;
        setDirtyBlockIndex.insert(pindex);
        setBlockIndexCandidates.erase(pindex);
        InvalidChainFound(pindex);
    }
}

bool Chainstate::ActivateBestChainStep(CValidationState& state, CBlockIndex* pindexMostWork,
                                       const std::shared_ptr<const CBlock>& pblock, bool& fInvalidFound,
                                       ConnectTrace& trace) {
    const CBlockIndex* pindexOldTip = chainActive.Tip();
    const CBlockIndex* pindexFork = chainActive.FindFork(pindexMostWork);
    bool fBlocksDisconnected = false;
    while (chainActive.Tip() && chainActive.Tip() != pindexFork) {
        if (!DisconnectTip(state)) return false;
        fBlocksDisconnected = true;
    }
    std::vector<CBlockIndex*> vpindexToConnect;
    bool fContinue = true;
    int nHeight = pindexFork ? pindexFork->nHeight : -1;
    while (fContinue && nHeight != pindexMostWork->nHeight) {
        // connect in batches of 32 so the tip (and RPC) progresses during long reorgs / IBD
        const int nTargetHeight = std::min(nHeight + 32, pindexMostWork->nHeight);
        vpindexToConnect.clear();
        CBlockIndex* pindexIter = pindexMostWork->GetAncestor(nTargetHeight);
        while (pindexIter && pindexIter->nHeight != nHeight) {
            vpindexToConnect.push_back(pindexIter);
            pindexIter = pindexIter->pprev;
        }
        nHeight = nTargetHeight;
        for (auto it = vpindexToConnect.rbegin(); it != vpindexToConnect.rend(); ++it) {
            CBlockIndex* pindexConnect = *it;
            const int64_t tTip = GetTimeMicros();
            // the block after this one, for the connect lookahead
            pindexConnectNext = pindexMostWork->nHeight > pindexConnect->nHeight
                                    ? pindexMostWork->GetAncestor(pindexConnect->nHeight + 1)
                                    : nullptr;
            const bool tipOk = ConnectTip(state, pindexConnect,
                                          pindexConnect == pindexMostWork ? pblock : std::shared_ptr<const CBlock>(), trace);
            pindexConnectNext = nullptr;
            phaseMicros[PH_ABC_TIP].fetch_add(GetTimeMicros() - tTip, std::memory_order_relaxed);
            if (!tipOk) {
                if (state.IsInvalid()) {
                    if (!state.CorruptionPossible()) InvalidChainFound(vpindexToConnect.front());
                    CheckForkWarningConditionsOnNewFork(vpindexToConnect.back());
                    state = CValidationState();
                    fInvalidFound = true;
                    fContinue = false;
                    trace.blocksConnected.pop_back();
                    break;
                }
                return false;
            }
            PruneBlockIndexCandidates();
            if (!pindexOldTip || chainActive.Tip()->nChainWork > pindexOldTip->nChainWork) {
                fContinue = false;
                break;
            }
        }
    }
    if (fBlocksDisconnected && mempool) {
        RemoveForReorgAtTip();
        LimitMempoolSize(gArgs.GetArg("-maxmempool", (int64_t)DEFAULT_MAX_MEMPOOL_SIZE) * 1000000,
                         gArgs.GetArg("-mempoolexpiry", (int64_t)DEFAULT_MEMPOOL_EXPIRY) * 60 * 60);
    }
    if (mempool) mempool->check(pcoinsTip.get(), chainActive.Height() + 1);
    // a new best chain re-evaluates the fork warnings (an invalid branch that is no longer 6+
    // blocks ahead clears them and leaves safe mode); reference validation.cpp:2758-2762
    if (!fInvalidFound) CheckForkWarningConditions();
    return true;
}

bool Chainstate::ActivateBestChain(CValidationState& state, std::shared_ptr<const CBlock> pblock) {
    CBlockIndex* pindexMostWork = nullptr;
    CBlockIndex* pindexNewTip = nullptr;
    int64_t tPh = GetTimeMicros();
    auto phase = [&](ConnectPhase ph) {
        const int64_t t = GetTimeMicros();
        phaseMicros[ph].fetch_add(t - tPh, std::memory_order_relaxed);
        tPh = t;
    };
    do {
        const CBlockIndex* pindexFork;
        bool fInitialDownload;
        ConnectTrace trace;
        {
            std::lock_guard<CCriticalSection> l(cs_main);
            CBlockIndex* pindexOldTip = chainActive.Tip();
            if (pindexMostWork == nullptr) pindexMostWork = FindMostWorkChain();
            phase(PH_ABC_FIND);
            if (pindexMostWork == nullptr || pindexMostWork == chainActive.Tip()) return true;
            bool fInvalidFound = false;
            std::shared_ptr<const CBlock> nullBlockPtr;
            if (!ActivateBestChainStep(state, pindexMostWork,
                                       pblock && pblock->GetHash(params.GetConsensus()) == pindexMostWork->GetBlockHash()
                                           ? pblock
                                           : nullBlockPtr,
                                       fInvalidFound, trace))
                return false;
            if (fInvalidFound) pindexMostWork = nullptr;
            pindexNewTip = chainActive.Tip();
            pindexFork = chainActive.FindFork(pindexOldTip);
            fInitialDownload = IsInitialBlockDownload();
            phase(PH_ABC_STEP);
            for (const auto& pb : trace.blocksConnected) {
                std::vector<CTransactionRef> conflicted;
                GetMainSignals().BlockConnected(pb.second, pb.first, conflicted);
            }
            phase(PH_ABC_SIGNALS);
        }
        // the connected blocks (a 7.5 MB block is ~100k heap objects) are freed on the reaper
        // thread, not between this block and the next (5-10 ms per block in IBD)
        Reaper::Get().Drop(std::move(trace.blocksConnected));
        phase(PH_ABC_REAP);
        if (pindexFork != pindexNewTip) {
            GetMainSignals().UpdatedBlockTip(pindexNewTip, pindexFork, fInitialDownload);
            uiInterface.NotifyBlockTip(fInitialDownload, pindexNewTip);
        }
        phase(PH_ABC_NOTIFY);
    } while (pindexNewTip != pindexMostWork);
    CheckBlockIndex(); // (takes cs_main)
    phase(PH_ABC_CHECKINDEX);
    const bool flushed = FlushStateToDisk(state, FLUSH_STATE_PERIODIC);
    phase(PH_ABC_FLUSH);
    return flushed;
}

bool Chainstate::PreciousBlock(CValidationState& state, CBlockIndex* pindex) {
    {
        std::lock_guard<CCriticalSection> l(cs_main);
        if (pindex->nChainWork < chainActive.Tip()->nChainWork) return true;
        if (chainActive.Tip()->nChainWork > nLastPreciousChainwork) nBlockReverseSequenceId = -1;
        nLastPreciousChainwork = chainActive.Tip()->nChainWork;
        setBlockIndexCandidates.erase(pindex);
        pindex->nSequenceId = nBlockReverseSequenceId;
        if (nBlockReverseSequenceId > std::numeric_limits<int32_t>::min()) nBlockReverseSequenceId--;
        if (pindex->IsValid(BLOCK_VALID_TRANSACTIONS) && pindex->nChainTx) {
            setBlockIndexCandidates.insert(pindex);
            PruneBlockIndexCandidates();
        }
    }
    return ActivateBestChain(state);
}

bool Chainstate::InvalidateBlock(CValidationState& state, CBlockIndex* pindex) {
    std::lock_guard<CCriticalSection> l(cs_main);
    pindex->nStatus |= BLOCK_FAILED_VALID;
    setDirtyBlockIndex.insert(pindex);
    setBlockIndexCandidates.erase(pindex);
    while (chainActive.Contains(pindex)) {
        CBlockIndex* pindexWalk = chainActive.Tip();
        pindexWalk->nStatus |= BLOCK_FAILED_CHILD;
        setDirtyBlockIndex.insert(pindexWalk);
        setBlockIndexCandidates.erase(pindexWalk);
        if (!DisconnectTip(state)) {
            if (mempool) RemoveForReorgAtTip();
            return false;
        }
    }
    LimitMempoolSize(gArgs.GetArg("-maxmempool", (int64_t)DEFAULT_MAX_MEMPOOL_SIZE) * 1000000,
                     gArgs.GetArg("-mempoolexpiry", (int64_t)DEFAULT_MEMPOOL_EXPIRY) * 60 * 60);
    // the chain tip may now be worse than other candidates: re-add everything better
    for (const auto& kv : mapBlockIndex) {
        CBlockIndex* p = kv.second;
        if (p->IsValid(BLOCK_VALID_TRANSACTIONS) && p->nChainTx && !setBlockIndexCandidates.value_comp()(p, chainActive.Tip()))
            setBlockIndexCandidates.insert(p);
    }
    InvalidChainFound(pindex);
    if (mempool) RemoveForReorgAtTip();
    return true;
}

// Drop mempool entries whose lock times or sequence locks no longer hold at the (new) tip. The
// callbacks run inside removeForReorg, still under the caller's cs_main.
void Chainstate::RemoveForReorgAtTip() {
    mempool->removeForReorg(
        pcoinsTip.get(), (unsigned)chainActive.Tip()->nHeight + 1, STANDARD_LOCKTIME_VERIFY_FLAGS,
        [&](const CTransaction& tx, LockPoints& lp, bool validLP) {
            AssertLockHeld(cs_main);
            CValidationState st;
            if (!ContextualCheckTransactionForCurrentBlock(tx, st, STANDARD_LOCKTIME_VERIFY_FLAGS)) return false;
            return CheckSequenceLocks(tx, STANDARD_LOCKTIME_VERIFY_FLAGS, &lp, validLP);
        },
        [&](const LockPoints* lp) {
            AssertLockHeld(cs_main);
            return TestLockPointValidity(lp);
        });
}

bool Chainstate::ResetBlockFailureFlags(CBlockIndex* pindex) {
    std::lock_guard<CCriticalSection> l(cs_main);
    const int nHeight = pindex->nHeight;
    for (const auto& kv : mapBlockIndex) {
        CBlockIndex* it = kv.second;
        if (!it->IsValid() && it->GetAncestor(nHeight) == pindex) {
            it->nStatus &= ~BLOCK_FAILED_MASK;
            setDirtyBlockIndex.insert(it);
            if (it->IsValid(BLOCK_VALID_TRANSACTIONS) && it->nChainTx &&
                setBlockIndexCandidates.value_comp()(chainActive.Tip(), it))
                setBlockIndexCandidates.insert(it);
            if (it == pindexBestInvalid) pindexBestInvalid = nullptr;
        }
    }
    while (pindex != nullptr) {
        if (pindex->nStatus & BLOCK_FAILED_MASK) {
            pindex->nStatus &= ~BLOCK_FAILED_MASK;
            setDirtyBlockIndex.insert(pindex);
        }
        pindex = pindex->pprev;
    }
    return true;
}

// ------------------------------------------------------------------ queries
bool Chainstate::IsInitialBlockDownload() const {
    if (latchToFalse.load(std::memory_order_relaxed)) return false;
    std::lock_guard<CCriticalSection> l(cs_main);
    if (latchToFalse.load(std::memory_order_relaxed)) return false;
    if (fReindex) return true;
    if (chainActive.Tip() == nullptr) return true;
    if (chainActive.Tip()->nChainWork < UintToArith256(params.GetConsensus().nMinimumChainWork)) return true;
    if (chainActive.Tip()->GetBlockTime() < (GetTime() - opts.maxTipAge)) return true;
    latchToFalse.store(true, std::memory_order_relaxed);
    return false;
}

CBlockIndex* Chainstate::FindForkInGlobalIndex(const CBlockLocator& locator) const {
    std::lock_guard<CCriticalSection> l(cs_main);
    for (const uint256& hash : locator.vHave) {
        CBlockIndex* pindex = LookupBlockIndex(hash);
        if (pindex) {
            if (chainActive.Contains(pindex)) return pindex;
            if (pindex->GetAncestor(chainActive.Height()) == chainActive.Tip()) return chainActive.Tip();
        }
    }
    return chainActive.Genesis();
}

std::vector<const CBlockIndex*> Chainstate::GetChainTips() const {
    std::lock_guard<CCriticalSection> l(cs_main);
    std::set<const CBlockIndex*> setOrphans, setPrevs;
    for (const auto& kv : mapBlockIndex) {
        if (!chainActive.Contains(kv.second)) {
            setOrphans.insert(kv.second);
            setPrevs.insert(kv.second->pprev);
        }
    }
    std::vector<const CBlockIndex*> tips;
    for (const CBlockIndex* p : setOrphans)
        if (setPrevs.erase(p) == 0) tips.push_back(p);
    tips.push_back(chainActive.Tip());
    std::sort(tips.begin(), tips.end(), [](const CBlockIndex* a, const CBlockIndex* b) { return a->nHeight > b->nHeight; });
    return tips;
}

double Chainstate::GuessVerificationProgress(const CBlockIndex* pindex) const {
    if (pindex == nullptr) return 0.0;
    const ChainTxData& data = params.TxData();
    const int64_t nNow = time(nullptr);
    double fTxTotal;
    if (pindex->nChainTx <= (unsigned)data.nTxCount) fTxTotal = (double)data.nTxCount + (nNow - data.nTime) * data.dTxRate;
    else fTxTotal = pindex->nChainTx + (nNow - pindex->GetBlockTime()) * data.dTxRate;
    return fTxTotal > 0 ? std::min(1.0, pindex->nChainTx / fTxTotal) : 1.0;
}

ThresholdState Chainstate::DeploymentState(const CBlockIndex* pindexPrev, Consensus::DeploymentPos pos) {
    return VersionBitsState(pindexPrev, params.GetConsensus(), pos, versionbitscache);
}
int32_t Chainstate::ComputeBlockVersion(const CBlockIndex* pindexPrev) {
    return bcp::ComputeBlockVersion(pindexPrev, params.GetConsensus(), versionbitscache);
}

void Chainstate::WaitForBlockChange(int64_t timeoutMillis, const uint256& from) {
    std::unique_lock<CCriticalSection> l(cs_main);
    AssertLockHeld(cs_main); // (unique_lock is invisible to the thread-safety analysis)
    auto pred = [&] {
        AssertLockHeld(cs_main); // evaluated by the wait with `l` held
        return chainActive.Tip() && chainActive.Tip()->GetBlockHash() != from;
    };
    if (timeoutMillis <= 0) cvBlockChange.wait(l, pred);
    else cvBlockChange.wait_for(l, std::chrono::milliseconds(timeoutMillis), pred);
}

bool Chainstate::GetTransaction(const uint256& txid, CTransactionRef& txOut, uint256& hashBlock, bool fAllowSlow) {
    std::lock_guard<CCriticalSection> l(cs_main);
    if (mempool) {
        CTransactionRef ptx = mempool->get(txid);
        if (ptx) {
            txOut = ptx;
            return true;
        }
    }
    if (opts.txindex) {
        CDiskTxPos postx;
        if (pblocktree->ReadTxIndex(txid, postx)) {
            CBlock block;
            CBlockIndex* found = nullptr;
            // locate the block by position
            for (const auto& kv : mapBlockIndex)
                if ((kv.second->nStatus & BLOCK_HAVE_DATA) && kv.second->nFile == postx.nFile &&
                    kv.second->nDataPos == postx.nPos) {
                    found = kv.second;
                    break;
                }
            if (found && ReadBlockFromDisk(block, found, params, false)) {
                for (const auto& tx : block.vtx)
                    if (tx->GetHash() == txid) {
                        txOut = tx;
                        hashBlock = found->GetBlockHash();
                        return true;
                    }
            }
        }
    }
    if (fAllowSlow) {
        const Coin& coin = AccessByTxid(*pcoinsTip, txid);
        CBlockIndex* pindexSlow = coin.IsSpent() ? nullptr : chainActive[coin.GetHeight()];
        if (pindexSlow) {
            CBlock block;
            if (ReadBlockFromDisk(block, pindexSlow, params, false)) {
                for (const auto& tx : block.vtx)
                    if (tx->GetHash() == txid) {
                        txOut = tx;
                        hashBlock = pindexSlow->GetBlockHash();
                        return true;
                    }
            }
        }
    }
    return false;
}

// ------------------------------------------------------------------ consistency checks
void Chainstate::CheckBlockIndex() {
    if (!opts.checkBlockIndex) return;
    std::lock_guard<CCriticalSection> l(cs_main);
    if (chainActive.Height() < 0) return;
    size_t nNodes = 0;
    for (const auto& kv : mapBlockIndex) {
        const CBlockIndex* p = kv.second;
        nNodes++;
        if (p->pprev == nullptr) {
            if (p->GetBlockHash() != params.GetConsensus().hashGenesisBlock)
                throw std::logic_error("CheckBlockIndex: orphan index entry " + p->GetBlockHash().ToString());
            continue;
        }
        if (p->nHeight != p->pprev->nHeight + 1) throw std::logic_error("CheckBlockIndex: height mismatch");
        if (p->nChainWork < p->pprev->nChainWork) throw std::logic_error("CheckBlockIndex: chainwork decreases");
        if (p->nTx > 0 && p->pprev->nChainTx > 0 && p->nChainTx != 0 && p->nChainTx != p->pprev->nChainTx + p->nTx)
            throw std::logic_error("CheckBlockIndex: nChainTx inconsistent");
        if ((p->nStatus & BLOCK_FAILED_MASK) == 0 && (p->pprev->nStatus & BLOCK_FAILED_MASK) != 0 &&
            chainActive.Contains(p))
            throw std::logic_error("CheckBlockIndex: valid child of invalid parent in active chain");
        if (p->pskip && p->pskip->nHeight >= p->nHeight) throw std::logic_error("CheckBlockIndex: bad skip");
    }
    for (const CBlockIndex* c : setBlockIndexCandidates)
        if (!c->IsValid(BLOCK_VALID_TRANSACTIONS) || !c->nChainTx)
            throw std::logic_error("CheckBlockIndex: candidate without data");
    (void)nNodes;
}

} // namespace bcp
