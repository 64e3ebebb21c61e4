#include "node/miner.h"
#include "node/gpuverify.h"

#include <thread>
#include "consensus/equihash.h"
#include "crypto/common.h"
#include "consensus/merkle.h"
#include "consensus/pow.h"
#include "kernels/gpu_api.h"
#include "keys/key.h"
#include "node/policy.h"
#include "node/txmempool.h"
#include "util/strencodings.h"

#include <algorithm>
#include <cassert>
#include <mutex>

namespace bcp {

uint64_t BlockAssembler::nLastBlockTx = 0;
uint64_t BlockAssembler::nLastBlockSize = 0;

static const unsigned MAX_COINBASE_SCRIPTSIG_SIZE = 100;

BlockAssembler::Options::Options()
    : nMaxGeneratedBlockSize((uint64_t)gArgs.GetArg("-blockmaxsize", (int64_t)DEFAULT_MAX_GENERATED_BLOCK_SIZE)),
      blockMinFeeRate(gArgs.IsArgSet("-blockmintxfee")
                          ? [] {
                                int64_t n = 0;
                                ParseMoney(gArgs.GetArg("-blockmintxfee", ""), n);
                                return CFeeRate(n);
                            }()
                          : CFeeRate(DEFAULT_BLOCK_MIN_TX_FEE)),
      nBlockPriorityPercentage(gArgs.GetArg("-blockprioritypercentage", (int64_t)DEFAULT_BLOCK_PRIORITY_PERCENTAGE)) {}

uint64_t ComputeMaxGeneratedBlockSize(uint64_t excessiveBlockSize) {
    // leave room for the coinbase; never exceed the excessive block size
    uint64_t n = (uint64_t)gArgs.GetArg("-blockmaxsize", (int64_t)DEFAULT_MAX_GENERATED_BLOCK_SIZE);
    n = std::max<uint64_t>(1000, std::min<uint64_t>(excessiveBlockSize - 1000, n));
    return n;
}

std::string GetSubVersionEB(uint64_t maxBlockSize) {
    // one decimal place of MB, e.g. 8000000 -> "8.0"
    const uint64_t tenths = maxBlockSize / 100000;
    return strprintf("%llu.%llu", (unsigned long long)(tenths / 10), (unsigned long long)(tenths % 10));
}

int64_t UpdateTime(CBlockHeader* pblock, const Consensus::Params& params, const CBlockIndex* pindexPrev) {
    const int64_t nOldTime = pblock->nTime;
    const int64_t nNewTime = std::max(pindexPrev->GetMedianTimePast() + 1, GetAdjustedTime());
    if (nOldTime < nNewTime) pblock->nTime = (uint32_t)nNewTime;
    // testnet: a late block may use minimum difficulty, which depends on the time
    if (params.fPowAllowMinDifficultyBlocks) pblock->nBits = GetNextWorkRequired(pindexPrev, pblock, params);
    return nNewTime - nOldTime;
}

BlockAssembler::BlockAssembler(Chainstate& cs, CTxMemPool* mp, const Options& o) : chainstate(cs), mempool(mp), options(o) {
    nMaxGeneratedBlockSize = std::max<uint64_t>(1000, std::min<uint64_t>(chainstate.MaxBlockSize() - 1000,
                                                                          options.nMaxGeneratedBlockSize));
    fPrintPriority = gArgs.GetBoolArg("-printpriority", false);
}

void BlockAssembler::resetBlock() {
    inBlock.clear();
    nBlockSize = 1000; // reserve space for the coinbase
    nBlockSigOps = 100;
    nBlockTx = 0;
    nFees = 0;
}

bool BlockAssembler::TestTxForBlock(const CTransaction& tx, uint64_t size, int64_t sigops) const {
    if (nBlockSize + size >= nMaxGeneratedBlockSize) return false;
    if (nBlockSigOps + sigops >= GetMaxBlockSigOpsCount(nBlockSize + size)) return false;
    CValidationState state;
    if (!chainstate.ContextualCheckTransaction(tx, state, nHeight, nLockTimeCutoff)) return false;
    return true;
}

void BlockAssembler::AddToBlock(const CTxMemPoolEntry& e) {
    const CTransactionRef& tx = e.GetSharedTx();
    pblock->vtx.push_back(tx);
    pblocktemplate->vTxFees.push_back(e.GetFee());
    pblocktemplate->vTxSigOpsCount.push_back(e.GetSigOpCount());
    nBlockSize += tx->GetTotalSize();
    ++nBlockTx;
    nBlockSigOps += e.GetSigOpCount();
    nFees += e.GetFee();
    inBlock.insert(tx->GetHash());
    if (fPrintPriority) { // reference miner.cpp:362-371
        double dPriority = e.GetPriority(nHeight);
        Amount dummy = 0;
        mempool->ApplyDeltas(tx->GetHash(), dPriority, dummy);
        LogPrintf("priority %.1f fee %s txid %s\n", dPriority, CFeeRate(e.GetModifiedFee(), e.GetTxSize()).ToString().c_str(),
                  tx->GetHash().ToString().c_str());
    }
}

void BlockAssembler::addPriorityTxs() {
    // a fraction of the block is reserved for high-priority (coin age) transactions
    if (options.nBlockPriorityPercentage == 0) return;
    const uint64_t nBlockPrioritySize = nMaxGeneratedBlockSize * options.nBlockPriorityPercentage / 100;
    std::vector<std::pair<double, const CTxMemPoolEntry*>> vecPriority;
    for (const CTxMemPoolEntry* e : mempool->SortedByDepthAndScore()) {
        double dPriority = e->GetPriority(nHeight);
        Amount dummy = 0;
        mempool->ApplyDeltas(e->GetTx().GetHash(), dPriority, dummy);
        vecPriority.push_back(std::make_pair(dPriority, e));
    }
    std::stable_sort(vecPriority.begin(), vecPriority.end(),
                     [](const std::pair<double, const CTxMemPoolEntry*>& a, const std::pair<double, const CTxMemPoolEntry*>& b) {
                         return a.first > b.first;
                     });
    bool progress = true;
    while (progress && nBlockSize < nBlockPrioritySize) {
        progress = false;
        for (const auto& p : vecPriority) {
            const CTxMemPoolEntry* e = p.second;
            const uint256& h = e->GetTx().GetHash();
            if (inBlock.count(h)) continue;
            if (!AllowFree(p.first)) return; // priority area closed below the free threshold
            bool dependent = false;
            for (const CTxIn& in : e->GetTx().vin)
                if (mempool->exists(in.prevout.hash) && !inBlock.count(in.prevout.hash)) dependent = true;
            if (dependent) continue;
            if (!TestTxForBlock(e->GetTx(), e->GetTxSize(), e->GetSigOpCount())) continue;
            AddToBlock(*e);
            progress = true;
            if (nBlockSize >= nBlockPrioritySize) return;
        }
    }
}

// Ancestor-feerate package selection: highest ancestor score first; each package is
// the candidate plus its not-yet-included ancestors, added in topological order.
void BlockAssembler::addPackageTxs() {
    std::vector<CTxMemPool::txiter> order = mempool->SortedByAncestorScore();
    int nConsecutiveFailed = 0;
    for (CTxMemPool::txiter it : order) {
        const CTxMemPoolEntry& e = *it->second;
        if (inBlock.count(it->first)) continue;
        std::vector<const CTxMemPoolEntry*> pkg = mempool->GetAncestors(it->first);
        pkg.erase(std::remove_if(pkg.begin(), pkg.end(),
                                 [&](const CTxMemPoolEntry* a) { return inBlock.count(a->GetTx().GetHash()) > 0; }),
                  pkg.end());
        pkg.push_back(&e);
        uint64_t pkgSize = 0;
        int64_t pkgSigOps = 0;
        Amount pkgFees = 0;
        for (const CTxMemPoolEntry* p : pkg) {
            pkgSize += p->GetTxSize();
            pkgSigOps += p->GetSigOpCount();
            pkgFees += p->GetModifiedFee();
        }
        if (pkgFees < options.blockMinFeeRate.GetFee(pkgSize)) break; // sorted: nothing better follows
        bool fits = nBlockSize + pkgSize < nMaxGeneratedBlockSize &&
                    nBlockSigOps + pkgSigOps < GetMaxBlockSigOpsCount(nBlockSize + pkgSize);
        if (fits) {
            for (const CTxMemPoolEntry* p : pkg)
                if (!TestTxForBlock(p->GetTx(), 0, 0)) fits = false;
        }
        if (!fits) {
            ++nConsecutiveFailed;
            if (nConsecutiveFailed > 1000 && nBlockSize > nMaxGeneratedBlockSize - 1000) break;
            continue;
        }
        std::sort(pkg.begin(), pkg.end(), [](const CTxMemPoolEntry* a, const CTxMemPoolEntry* b) {
            if (a->GetCountWithAncestors() != b->GetCountWithAncestors())
                return a->GetCountWithAncestors() < b->GetCountWithAncestors();
            return a->GetTx().GetHash() < b->GetTx().GetHash();
        });
        for (const CTxMemPoolEntry* p : pkg) AddToBlock(*p);
        nConsecutiveFailed = 0;
    }
}

std::unique_ptr<CBlockTemplate> BlockAssembler::CreateNewBlock(const CScript& scriptPubKeyIn) {
    const int64_t nTimeStart = GetTimeMicros();
    resetBlock();
    pblocktemplate.reset(new CBlockTemplate());
    pblock = &pblocktemplate->block;
    pblock->vtx.emplace_back();
    pblocktemplate->vTxFees.push_back(-1);
    pblocktemplate->vTxSigOpsCount.push_back(-1);
    std::lock_guard<CCriticalSection> l(chainstate.cs());
    // cs_main then the mempool lock for the whole template, like the reference's LOCK2; without a
    // mempool (tests) a private lock stands in so the scope stays unconditional
    static CCriticalSection noMempool{"miner.nomempool"};
    std::lock_guard<CCriticalSection> lmp(mempool ? mempool->cs : noMempool);
    const CChainParams& chainparams = chainstate.Params();
    const Consensus::Params& cp = chainparams.GetConsensus();
    CBlockIndex* pindexPrev = chainstate.Tip();
    nHeight = pindexPrev->nHeight + 1;
    pblock->nVersion = chainstate.ComputeBlockVersion(pindexPrev);
    if (chainparams.MineBlocksOnDemand()) pblock->nVersion = (int32_t)gArgs.GetArg("-blockversion", (int64_t)pblock->nVersion);
    pblock->nTime = (uint32_t)GetAdjustedTime();
    nLockTimeCutoff = (STANDARD_LOCKTIME_VERIFY_FLAGS & LOCKTIME_MEDIAN_TIME_PAST) ? pindexPrev->GetMedianTimePast()
                                                                                   : pblock->GetBlockTime();
    if (mempool) {
        addPriorityTxs();
        addPackageTxs();
    }
    nLastBlockTx = nBlockTx;
    nLastBlockSize = nBlockSize;

    CMutableTransaction coinbaseTx;
    coinbaseTx.vin.resize(1);
    coinbaseTx.vin[0].prevout.SetNull();
    coinbaseTx.vout.resize(1);
    coinbaseTx.vout[0].scriptPubKey = scriptPubKeyIn;
    coinbaseTx.vout[0].nValue = nFees + GetBlockSubsidy(nHeight, cp);
    coinbaseTx.vin[0].scriptSig = CScript() << nHeight << OP_0;
    pblock->vtx[0] = MakeTransactionRef(std::move(coinbaseTx));
    pblocktemplate->vTxFees[0] = -1 * nFees;

    arith_uint256 nonce;
    if (nHeight >= cp.BCPHeight) {
        // random 256-bit nonce; top and bottom 16 bits cleared for local counters/flags
        nonce = UintToArith256(GetRandHash());
        nonce <<= 32;
        nonce >>= 16;
    }
    pblock->hashPrevBlock = pindexPrev->GetBlockHash();
    pblock->nHeight = (uint32_t)nHeight;
    memset(pblock->nReserved, 0, sizeof(pblock->nReserved));
    UpdateTime(pblock, cp, pindexPrev);
    pblock->nBits = GetNextWorkRequired(pindexPrev, pblock, cp);
    pblock->nNonce = ArithToUint256(nonce);
    pblock->nSolution.clear();
    pblocktemplate->vTxSigOpsCount[0] = (int64_t)GetSigOpCountWithoutP2SH(*pblock->vtx[0]);
    pblock->hashMerkleRoot = BlockMerkleRoot(*pblock);

    CValidationState state;
    if (!chainstate.TestBlockValidity(state, *pblock, pindexPrev, false, false))
        throw std::runtime_error(strprintf("CreateNewBlock: TestBlockValidity failed: %s", FormatStateMessage(state).c_str()));
    LogPrint(BCLog::BENCH, "CreateNewBlock(): %u txs, fees %lld, %.2fms\n", (unsigned)nBlockTx, (long long)nFees,
             0.001 * (GetTimeMicros() - nTimeStart));
    return std::move(pblocktemplate);
}

void IncrementExtraNonce(CBlock* pblock, const CBlockIndex* pindexPrev, unsigned& nExtraNonce, uint64_t maxBlockSize) {
    static uint256 hashPrevBlock;
    static std::mutex m;
    {
        std::lock_guard<std::mutex> l(m);
        if (hashPrevBlock != pblock->hashPrevBlock) {
            nExtraNonce = 0;
            hashPrevBlock = pblock->hashPrevBlock;
        }
    }
    ++nExtraNonce;
    const int nHeight = pindexPrev->nHeight + 1;
    CMutableTransaction txCoinbase(*pblock->vtx[0]);
    const std::string eb = "/EB" + GetSubVersionEB(maxBlockSize) + "/";
    txCoinbase.vin[0].scriptSig = CScript() << nHeight << CScriptNum((int64_t)nExtraNonce)
                                            << std::vector<unsigned char>(eb.begin(), eb.end());
    if (txCoinbase.vin[0].scriptSig.size() > MAX_COINBASE_SCRIPTSIG_SIZE) throw std::logic_error("coinbase scriptSig too large");
    pblock->vtx[0] = MakeTransactionRef(std::move(txCoinbase));
    pblock->hashMerkleRoot = BlockMerkleRoot(*pblock);
}

// ------------------------------------------------------------------ PoW search
static std::mutex g_minerMutex;
static MinerStats g_minerStats;
MinerStats GetMinerStats() {
    std::lock_guard<std::mutex> l(g_minerMutex);
    return g_minerStats;
}

namespace {
// Two solvers per (device, N, K), kept across blocks: (200,9) at batch 32 holds ~17 GiB each
// (one slot array per stage, csrc/kernels/equihash_solver.hip).
struct DeviceMiner {
    int device;
    unsigned n, k;
    std::mutex busy;
    std::unique_ptr<gpu::EquihashGpuSolver> s[2];
};
std::mutex g_devMinersMutex;
std::vector<std::unique_ptr<DeviceMiner>> g_devMiners;
std::vector<int> g_minerDevices;

DeviceMiner& GetDeviceMiner(int device, unsigned n, unsigned k) {
    std::lock_guard<std::mutex> l(g_devMinersMutex);
    for (auto& d : g_devMiners)
        if (d->device == device && d->n == n && d->k == k) return *d;
    std::unique_ptr<DeviceMiner> d(new DeviceMiner);
    d->device = device;
    d->n = n;
    d->k = k;
    const int batch = n == 200 ? 32 : 16;
    for (auto& s : d->s) s.reset(new gpu::EquihashGpuSolver(n, k, batch, device));
    g_devMiners.push_back(std::move(d));
    return *g_devMiners.back();
}
} // namespace

void SetMinerGpuDevices(const std::vector<int>& devices) {
    std::lock_guard<std::mutex> l(g_devMinersMutex);
    g_minerDevices = devices;
}
std::vector<int> GetMinerGpuDevices() {
    std::vector<int> d;
    {
        std::lock_guard<std::mutex> l(g_devMinersMutex);
        d = g_minerDevices;
    }
    if (d.empty()) {
        // default: every visible device except the explicitly configured validation devices,
        // unless that would leave none (then the miner shares them; validation lanes run at the
        // device's greatest stream priority, csrc/node/gpuverify.h)
        const std::vector<int> val = GpuVerifyService::Instance().ConfiguredDevices();
        const int cnt = gpu::DeviceCount();
        for (int i = 0; i < cnt; i++)
            if (std::find(val.begin(), val.end(), i) == val.end()) d.push_back(i);
        if (d.empty())
            for (int i = 0; i < cnt; i++) d.push_back(i);
    }
    return d;
}

EhSearchResult EquihashSearchGpu(unsigned n, unsigned k, const std::vector<unsigned char>& equihashInput,
                                 const uint256& nonce0, uint64_t maxNonces,
                                 const std::function<bool(const uint256&, const std::vector<unsigned char>&)>& accept,
                                 std::vector<int> devices, const std::atomic<bool>* cancel) {
    if (devices.empty()) devices = GetMinerGpuDevices();
    if (devices.empty()) throw std::runtime_error("EquihashSearchGpu: no GPU device");
    const EquihashParams ep(n, k);
    CBlake2b base = EhInitialiseState(ep);
    base.Write(equihashInput.data(), equihashInput.size());
    const arith_uint256 n0 = UintToArith256(nonce0);
    std::atomic<uint64_t> next{0}, nNonces{0}, nSols{0};
    std::atomic<bool> stop{false};
    std::mutex resMutex;
    EhSearchResult res;
    std::string firstError;
    auto worker = [&](int device) {
        try {
            DeviceMiner& dm = GetDeviceMiner(device, n, k);
            std::lock_guard<std::mutex> busy(dm.busy);
            const int B = dm.s[0]->Batch();
            std::vector<uint256> pend[2];
            auto launch = [&](int slot) -> bool {
                if (stop.load() || (cancel && cancel->load())) return false;
                const uint64_t start = next.fetch_add((uint64_t)B);
                if (start >= maxNonces) return false;
                const int nb = (int)std::min<uint64_t>((uint64_t)B, maxNonces - start);
                std::vector<gpu::EhBaseState> states(nb);
                pend[slot].resize(nb);
                for (int b = 0; b < nb; b++) {
                    pend[slot][b] = ArithToUint256(n0 + arith_uint256(start + 1 + (uint64_t)b));
                    CBlake2b st = base;
                    st.Write(pend[slot][b].begin(), 32);
                    states[b] = gpu::MakeEhBaseState(st);
                }
                dm.s[slot]->Launch(states);
                return true;
            };
            auto collect = [&](int slot) {
                const auto sols = dm.s[slot]->Collect();
                nNonces += pend[slot].size();
                for (size_t b = 0; b < sols.size(); b++)
                    for (const auto& idx : sols[b]) {
                        nSols++;
                        if (stop.load()) continue;
                        std::vector<unsigned char> minimal = GetMinimalFromIndices(idx, ep.N / (ep.K + 1));
                        if (!accept(pend[slot][b], minimal)) continue;
                        std::lock_guard<std::mutex> l(resMutex);
                        if (!res.found) {
                            res.found = true;
                            res.nonce = pend[slot][b];
                            res.solution = std::move(minimal);
                        }
                        stop = true;
                    }
            };
            bool inflight[2] = {launch(0), false};
            for (int cur = 0;; cur ^= 1) { // launch the next batch, then decode the running one
                inflight[cur ^ 1] = launch(cur ^ 1);
                if (inflight[cur]) collect(cur);
                inflight[cur] = false;
                if (!inflight[cur ^ 1]) break;
            }
        } catch (const std::exception& e) {
            std::lock_guard<std::mutex> l(resMutex);
            if (firstError.empty()) firstError = e.what();
            stop = true;
        }
    };
    std::vector<std::thread> threads;
    for (int d : devices) threads.emplace_back(worker, d);
    for (auto& t : threads) t.join();
    res.nonces = nNonces.load();
    res.solutions = nSols.load();
    if (!res.found && !firstError.empty()) throw std::runtime_error("EquihashSearchGpu: " + firstError);
    return res;
}

static bool SolveLegacy(CBlock& block, const Consensus::Params& cp, uint64_t& nMaxTries, bool useGpu,
                        const std::atomic<bool>* cancel) {
    // nonce lives in the low 32 bits of nNonce in the 80-byte legacy header
    uint32_t n32 = ReadLE32(block.nNonce.begin());
    // cheap CPU attempts first: regtest/min-difficulty targets pass almost immediately
    for (int i = 0; i < 4096 && nMaxTries > 0; i++) {
        if (CheckProofOfWork(block.GetHash(cp), block.nBits, false, cp)) return true;
        if (cancel && cancel->load()) return false;
        if (++n32 == 0) block.nTime++;
        WriteLE32(block.nNonce.begin(), n32);
        --nMaxTries;
        std::lock_guard<std::mutex> l(g_minerMutex);
        g_minerStats.sha_nonces++;
    }
    if (!useGpu || !gpu::GpuAvailable()) {
        while (nMaxTries > 0) {
            if (CheckProofOfWork(block.GetHash(cp), block.nBits, false, cp)) return true;
            if (cancel && cancel->load()) return false;
            if (++n32 == 0) block.nTime++; // nonce space wrapped: new header
            WriteLE32(block.nNonce.begin(), n32);
            --nMaxTries;
        }
        return false;
    }
    arith_uint256 target;
    target.SetCompact(block.nBits);
    const uint256 t = ArithToUint256(target);
    // Scan [n32, 2^32) in chunks; when the 32-bit nonce space is used up, bump nTime (a new
    // header) and start again from 0, so no nonce is scanned twice for the same header.
    const uint64_t NONCE_SPACE = 1ull << 32;
    while (nMaxTries > 0) {
        std::vector<unsigned char> hdr = SerializeToBytes(static_cast<const CBlockHeader&>(block), SER_NETWORK,
                                                          PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY);
        const uint64_t count = std::min<uint64_t>({nMaxTries, 1ull << 30, NONCE_SPACE - n32});
        const int64_t t0 = GetTimeMicros();
        const int64_t found = gpu::Sha256dScanNonces(hdr.data(), t.begin(), n32, count);
        const uint64_t scanned = found >= 0 ? (uint64_t)found - n32 + 1 : count;
        {
            std::lock_guard<std::mutex> l(g_minerMutex);
            g_minerStats.gpu_ms += (GetTimeMicros() - t0) / 1000.0;
            g_minerStats.sha_nonces += scanned;
        }
        nMaxTries -= std::min<uint64_t>(nMaxTries, scanned);
        if (found >= 0) {
            WriteLE32(block.nNonce.begin(), (uint32_t)found);
            if (CheckProofOfWork(block.GetHash(cp), block.nBits, false, cp)) return true;
            LogPrintf("SolveLegacy: GPU nonce %u failed the CPU proof-of-work recheck; scanning on\n",
                      (uint32_t)found);
        }
        const uint64_t next = (uint64_t)n32 + scanned;
        if (next >= NONCE_SPACE) {
            block.nTime++;
            n32 = 0;
        } else {
            n32 = (uint32_t)next;
        }
        WriteLE32(block.nNonce.begin(), n32);
        if (cancel && cancel->load()) return false;
    }
    return false;
}

static bool SolveEquihash(CBlock& block, const CChainParams& params, uint64_t& nMaxTries, bool useGpu,
                          const std::atomic<bool>* cancel) {
    const Consensus::Params& cp = params.GetConsensus();
    const EquihashParams ep(params.EquihashN(), params.EquihashK());
    CBlake2b base = EhInitialiseState(ep);
    const std::vector<unsigned char> input = block.EquihashInput();
    base.Write(input.data(), input.size());
    auto tryState = [&](const std::vector<unsigned char>& soln) {
        block.nSolution = soln;
        return CheckProofOfWork(block.GetHash(cp), block.nBits, true, cp);
    };
    const bool gpuOk = useGpu && gpu::GpuAvailable(); // (48,5) too: 0.086 vs 0.109 ms per nonce batch, profiles/baseline_metrics_r2s4.md
    if (gpuOk) {
        const CBlockHeader hdr = block.GetBlockHeader();
        auto accept = [&](const uint256& nonce, const std::vector<unsigned char>& soln) {
            CBlockHeader h = hdr; // thread-safe: each candidate hashes its own copy
            h.nNonce = nonce;
            h.nSolution = soln;
            return CheckProofOfWork(h.GetHash(cp), h.nBits, true, cp);
        };
        const int64_t t0 = GetTimeMicros();
        const EhSearchResult r = EquihashSearchGpu(ep.N, ep.K, input, block.nNonce, nMaxTries, accept, {}, cancel);
        {
            std::lock_guard<std::mutex> ls(g_minerMutex);
            g_minerStats.gpu_ms += (GetTimeMicros() - t0) / 1000.0;
            g_minerStats.eh_nonces += r.nonces;
            g_minerStats.eh_solutions += r.solutions;
        }
        nMaxTries -= std::min(nMaxTries, r.nonces);
        if (r.found) {
            block.nNonce = r.nonce;
            block.nSolution = r.solution;
            return true;
        }
        block.nNonce = ArithToUint256(UintToArith256(block.nNonce) + arith_uint256(r.nonces));
        return false;
    }
    while (nMaxTries > 0) {
        block.nNonce = ArithToUint256(UintToArith256(block.nNonce) + 1);
        CBlake2b st = base;
        st.Write(block.nNonce.begin(), 32);
        --nMaxTries;
        {
            std::lock_guard<std::mutex> ls(g_minerMutex);
            g_minerStats.eh_nonces++;
        }
        if (EhBasicSolve(ep, st, tryState, [&] { return cancel && cancel->load(); })) return true;
        if (cancel && cancel->load()) return false;
    }
    return false;
}

bool SolveBlock(CBlock& block, const CChainParams& params, uint64_t& nMaxTries, bool useGpu,
                const std::atomic<bool>* cancel) {
    const bool ok = (int)block.nHeight < params.GetConsensus().BCPHeight
                        ? SolveLegacy(block, params.GetConsensus(), nMaxTries, useGpu, cancel)
                        : SolveEquihash(block, params, nMaxTries, useGpu, cancel);
    if (ok) {
        std::lock_guard<std::mutex> l(g_minerMutex);
        g_minerStats.blocks++;
    }
    return ok;
}

std::vector<uint256> GenerateBlocks(Chainstate& chainstate, CTxMemPool* mempool, const CScript& coinbaseScript,
                                    int nGenerate, uint64_t nMaxTries, bool useGpu, std::string* err) {
    std::vector<uint256> hashes;
    int nHeight, nHeightEnd;
    {
        std::lock_guard<CCriticalSection> l(chainstate.cs());
        nHeight = chainstate.Height();
        nHeightEnd = nHeight + nGenerate;
    }
    unsigned nExtraNonce = 0;
    const CChainParams& params = chainstate.Params();
    while (nHeight < nHeightEnd) {
        std::unique_ptr<CBlockTemplate> tmpl = BlockAssembler(chainstate, mempool).CreateNewBlock(coinbaseScript);
        CBlock* pblock = &tmpl->block;
        {
            std::lock_guard<CCriticalSection> l(chainstate.cs());
            IncrementExtraNonce(pblock, chainstate.Tip(), nExtraNonce, chainstate.MaxBlockSize());
        }
        if (!SolveBlock(*pblock, params, nMaxTries, useGpu)) {
            if (nMaxTries == 0) break;
            continue;
        }
        auto shared = std::make_shared<const CBlock>(*pblock);
        CValidationState state;
        if (!chainstate.ProcessNewBlock(shared, true, nullptr, &state)) {
            if (err) *err = "ProcessNewBlock, block not accepted: " + FormatStateMessage(state);
            return hashes;
        }
        ++nHeight;
        hashes.push_back(pblock->GetHash(params.GetConsensus()));
    }
    return hashes;
}

} // namespace bcp
