// Chainstate loading, replay, verification, reindex/import and pruning.
// Parity: reference src/validation.cpp LoadBlockIndexDB :4033, CVerifyDB::VerifyDB :4167,
// RewindBlockIndex :4324, InitBlockIndex :4412, LoadExternalBlockFile :4461,
// FindFilesToPrune :3914, PruneOneBlockFile :3831, and the ReplayBlocks crash-recovery
// of the head-blocks marker written by CCoinsViewDB::BatchWrite.
#include "node/validation.h"
#include "node/ui_interface.h"
#include "consensus/pow.h"
#include "node/signals.h"
#include "util/strencodings.h"

#include <algorithm>
#include <deque>
#include <unistd.h>

namespace bcp {

bool Chainstate::LoadBlockIndexDB(std::string& err) {
    auto insert = [this](const uint256& h) {
        AssertLockHeld(cs_main); // called back synchronously from LoadBlockIndexGuts
        return InsertBlockIndex(h);
    };
    if (!pblocktree->LoadBlockIndexGuts(insert, params.GetConsensus())) {
        err = "Error loading block index (corrupt entry)";
        return false;
    }
    std::vector<std::pair<int, CBlockIndex*>> vSortedByHeight;
    vSortedByHeight.reserve(mapBlockIndex.size());
    for (const auto& item : mapBlockIndex) vSortedByHeight.push_back(std::make_pair(item.second->nHeight, item.second));
    std::sort(vSortedByHeight.begin(), vSortedByHeight.end());
    for (const auto& item : vSortedByHeight) {
        CBlockIndex* pindex = item.second;
        pindex->nChainWork = (pindex->pprev ? pindex->pprev->nChainWork : arith_uint256(0)) + GetBlockProof(*pindex);
        pindex->nTimeMax = pindex->pprev ? std::max(pindex->pprev->nTimeMax, pindex->nTime) : pindex->nTime;
        if (pindex->nTx > 0) {
            if (pindex->pprev) {
                if (pindex->pprev->nChainTx) {
                    pindex->nChainTx = pindex->pprev->nChainTx + pindex->nTx;
                } else {
                    pindex->nChainTx = 0;
                    mapBlocksUnlinked.insert(std::make_pair(pindex->pprev, pindex));
                }
            } else {
                pindex->nChainTx = pindex->nTx;
            }
        }
        if (pindex->IsValid(BLOCK_VALID_TRANSACTIONS) && (pindex->nChainTx || pindex->pprev == nullptr))
            setBlockIndexCandidates.insert(pindex);
        if ((pindex->nStatus & BLOCK_FAILED_MASK) &&
            (!pindexBestInvalid || pindex->nChainWork > pindexBestInvalid->nChainWork))
            pindexBestInvalid = pindex;
        if (pindex->pprev) pindex->BuildSkip();
        if (pindex->IsValid(BLOCK_VALID_TREE) &&
            (pindexBestHeader == nullptr || WorkComparator()(pindexBestHeader, pindex)))
            pindexBestHeader = pindex;
    }
    pblocktree->ReadLastBlockFile(nLastBlockFile);
    vinfoBlockFile.resize(nLastBlockFile + 1);
    for (int nFile = 0; nFile <= nLastBlockFile; nFile++) pblocktree->ReadBlockFileInfo(nFile, vinfoBlockFile[nFile]);
    for (int nFile = nLastBlockFile + 1;; nFile++) {
        CBlockFileInfo info;
        if (!pblocktree->ReadBlockFileInfo(nFile, info)) break;
        vinfoBlockFile.push_back(info);
    }
    std::set<int> setBlkDataFiles;
    for (const auto& item : mapBlockIndex)
        if (item.second->nStatus & BLOCK_HAVE_DATA) setBlkDataFiles.insert(item.second->nFile);
    for (int f : setBlkDataFiles) {
        FILE* fp = OpenBlockFile(CDiskBlockPos(f, 0), true);
        if (!fp) {
            err = strprintf("Missing block file blk%05u.dat", (unsigned)f);
            return false;
        }
        fclose(fp);
    }
    pblocktree->ReadFlag("prunedblockfiles", fHavePruned);
    bool fReindexing = false;
    pblocktree->ReadReindexing(fReindexing);
    fReindex |= fReindexing;
    bool txindex = opts.txindex;
    if (pblocktree->ReadFlag("txindex", txindex) && txindex != opts.txindex && !mapBlockIndex.empty()) {
        err = "You need to rebuild the database using -reindex to change -txindex";
        return false;
    }
    return true;
}

bool Chainstate::LoadChainTip() {
    auto it = mapBlockIndex.find(pcoinsTip->GetBestBlock());
    if (it == mapBlockIndex.end()) return false;
    chainActive.SetTip(it->second);
    PruneBlockIndexCandidates();
    LogPrintf("Loaded best chain: hashBestChain=%s height=%d\n", chainActive.Tip()->GetBlockHash().ToString().c_str(),
              chainActive.Height());
    return true;
}

bool Chainstate::LoadBlockIndex(std::string& err) {
    std::lock_guard<CCriticalSection> l(cs_main);
    if (fReindex) return true;
    if (!LoadBlockIndexDB(err)) return false;
    if (!mapBlockIndex.empty()) {
        if (!ReplayBlocks(err)) return false;
        if (!LoadChainTip() && !pcoinsTip->GetBestBlock().IsNull()) {
            err = "Coins database best block not found in block index";
            return false;
        }
    }
    return true;
}

bool Chainstate::InitBlockIndex(std::string& err) {
    std::lock_guard<CCriticalSection> l(cs_main);
    if (chainActive.Genesis() != nullptr) return true;
    pblocktree->WriteFlag("txindex", opts.txindex);
    try {
        const CBlock& block = params.GenesisBlock();
        CValidationState state;
        CDiskBlockPos blockPos;
        const unsigned nBlockSize = (unsigned)GetSerializeSize(block, PROTOCOL_VERSION);
        if (!FindBlockPos(state, blockPos, nBlockSize + 8, 0, block.GetBlockTime())) {
            err = "LoadBlockIndex(): FindBlockPos failed";
            return false;
        }
        if (!WriteBlockToDisk(block, blockPos, params.DiskMagic())) {
            err = "LoadBlockIndex(): writing genesis block to disk failed";
            return false;
        }
        CBlockIndex* pindex = AddToBlockIndex(block);
        if (!ReceivedBlockTransactions(block, state, pindex, blockPos)) {
            err = "LoadBlockIndex(): genesis block not accepted";
            return false;
        }
        if (!FlushStateToDisk(state, FLUSH_STATE_ALWAYS)) {
            err = "LoadBlockIndex(): flush failed";
            return false;
        }
        CValidationState st2;
        if (!ActivateBestChain(st2, std::make_shared<CBlock>(block))) {
            err = "LoadBlockIndex(): genesis activation failed: " + FormatStateMessage(st2);
            return false;
        }
    } catch (const std::runtime_error& e) {
        err = std::string("LoadBlockIndex(): failed to initialize block database: ") + e.what();
        return false;
    }
    return true;
}

// An interrupted UTXO flush leaves a head-blocks marker [new, old]: roll the coins from
// `old` forward to `new` by disconnecting back to the fork point and reconnecting.
bool Chainstate::ReplayBlocks(std::string& err) {
    std::lock_guard<CCriticalSection> l(cs_main); // startup, but DisconnectBlock expects the lock
    std::vector<uint256> heads = pcoinsdbview->GetHeadBlocks();
    if (heads.empty()) return true;
    if (heads.size() != 2) {
        err = "ReplayBlocks(): unknown inconsistent state";
        return false;
    }
    CCoinsViewCache cache(pcoinsdbview.get());
    const CBlockIndex* pindexNew = LookupBlockIndex(heads[0]);
    const CBlockIndex* pindexOld = heads[1].IsNull() ? nullptr : LookupBlockIndex(heads[1]);
    if (!pindexNew) {
        err = "ReplayBlocks(): reorganization to unknown block requested";
        return false;
    }
    const CBlockIndex* pindexFork = pindexOld ? LastCommonAncestor(pindexOld, pindexNew) : nullptr;
    while (pindexOld != pindexFork) {
        if (pindexOld->nHeight > 0) {
            CBlock block;
            if (!ReadBlockFromDisk(block, pindexOld, params)) {
                err = "ReplayBlocks(): failed to read block";
                return false;
            }
            if (DisconnectBlock(block, pindexOld, cache) == DISCONNECT_FAILED) {
                err = "ReplayBlocks(): disconnect failed";
                return false;
            }
        }
        pindexOld = pindexOld->pprev;
    }
    const int nForkHeight = pindexFork ? pindexFork->nHeight : 0;
    for (int nHeight = nForkHeight + 1; nHeight <= pindexNew->nHeight; ++nHeight) {
        const CBlockIndex* pindex = pindexNew->GetAncestor(nHeight);
        CBlock block;
        if (!ReadBlockFromDisk(block, pindex, params)) {
            err = "ReplayBlocks(): failed to read block";
            return false;
        }
        // outputs/spends only: scripts were validated before the interrupted flush
        for (const auto& tx : block.vtx) {
            if (!tx->IsCoinBase())
                for (const CTxIn& in : tx->vin) cache.SpendCoin(in.prevout);
            AddCoins(cache, *tx, pindex->nHeight, true);
        }
    }
    cache.SetBestBlock(pindexNew->GetBlockHash());
    cache.Flush();
    return true;
}

bool Chainstate::RewindBlockIndex() {
    // Blocks validated under rules that changed (none in this chain's history): only
    // verify that every connected block still carries BLOCK_VALID_SCRIPTS and undo data.
    std::lock_guard<CCriticalSection> l(cs_main);
    for (int h = 1; h <= chainActive.Height(); h++) {
        CBlockIndex* p = chainActive[h];
        if (!(p->nStatus & BLOCK_HAVE_UNDO) && !PruneMode()) {
            CValidationState state;
            while (chainActive.Height() >= h)
                if (!DisconnectTip(state, true)) return false;
            break;
        }
    }
    CValidationState state;
    return FlushStateToDisk(state, FLUSH_STATE_ALWAYS);
}

bool Chainstate::VerifyDB(int nCheckLevel, int nCheckDepth) {
    std::lock_guard<CCriticalSection> l(cs_main);
    if (chainActive.Tip() == nullptr || chainActive.Tip()->pprev == nullptr) return true;
    if (nCheckDepth <= 0 || nCheckDepth > chainActive.Height()) nCheckDepth = chainActive.Height();
    nCheckLevel = std::max(0, std::min(4, nCheckLevel));
    LogPrintf("Verifying last %i blocks at level %i\n", nCheckDepth, nCheckLevel);
    CCoinsViewCache coins(pcoinsTip.get());
    CBlockIndex* pindexState = chainActive.Tip();
    CBlockIndex* pindexFailure = nullptr;
    int nGoodTransactions = 0;
    CValidationState state;
    struct ProgressDone {
        ~ProgressDone() { uiInterface.ShowProgress("", 100); }
    } progressDone;
    uiInterface.ShowProgress("Verifying blocks...", 0);
    for (CBlockIndex* pindex = chainActive.Tip(); pindex && pindex->pprev; pindex = pindex->pprev) {
        const int pct = std::max(1, std::min(99, (int)(((double)(chainActive.Height() - pindex->nHeight)) /
                                                        (double)nCheckDepth * (nCheckLevel >= 4 ? 50 : 100))));
        uiInterface.ShowProgress("Verifying blocks...", pct);
        if (pindex->nHeight < chainActive.Height() - nCheckDepth) break;
        if (PruneMode() && !(pindex->nStatus & BLOCK_HAVE_DATA)) break;
        CBlock block;
        // level 0: read from disk
        if (!ReadBlockFromDisk(block, pindex, params)) return error("VerifyDB(): *** ReadBlockFromDisk failed");
        // level 1: verify block validity
        if (nCheckLevel >= 1 && !CheckBlock(block, state)) return error("VerifyDB(): *** found bad block");
        // level 2: verify undo validity
        if (nCheckLevel >= 2 && pindex) {
            CBlockUndo undo;
            CDiskBlockPos pos = pindex->GetUndoPos();
            if (!pos.IsNull() && !UndoReadFromDisk(undo, pos, pindex->pprev->GetBlockHash()))
                return error("VerifyDB(): *** found bad undo data");
        }
        // level 3: disconnect while the cache stays small
        if (nCheckLevel >= 3 && pindex == pindexState &&
            coins.DynamicMemoryUsage() + pcoinsTip->DynamicMemoryUsage() <= opts.coinsCacheBytes) {
            const DisconnectResult res = DisconnectBlock(block, pindex, coins);
            if (res == DISCONNECT_FAILED) return error("VerifyDB(): *** irrecoverable inconsistency");
            pindexState = pindex->pprev;
            if (res == DISCONNECT_UNCLEAN) {
                nGoodTransactions = 0;
                pindexFailure = pindex;
            } else {
                nGoodTransactions += (int)block.vtx.size();
            }
        }
    }
    if (pindexFailure)
        return error("VerifyDB(): *** coin database inconsistencies found (last %i blocks, %i good transactions before "
                     "that)",
                     chainActive.Height() - pindexFailure->nHeight + 1, nGoodTransactions);
    // level 4: reconnect the disconnected blocks
    if (nCheckLevel >= 4) {
        CBlockIndex* pindex = pindexState;
        while (pindex != chainActive.Tip()) {
            uiInterface.ShowProgress("Verifying blocks...",
                                     std::max(1, std::min(99, 100 - (int)(((double)(chainActive.Height() - pindex->nHeight)) /
                                                                          (double)nCheckDepth * 50))));
            pindex = chainActive.Next(pindex);
            CBlock block;
            if (!ReadBlockFromDisk(block, pindex, params)) return error("VerifyDB(): *** ReadBlockFromDisk failed");
            if (!ConnectBlock(block, state, pindex, coins)) return error("VerifyDB(): *** found unconnectable block");
        }
    }
    LogPrintf("No coin database inconsistencies in last %i blocks (%i transactions)\n",
              chainActive.Height() - pindexState->nHeight, nGoodTransactions);
    return true;
}

// Import blocks from a raw blk*.dat stream: scan for the disk magic, accept in order,
// defer out-of-order blocks until their parent arrives.
bool Chainstate::LoadExternalBlockFile(FILE* fileIn, CDiskBlockPos* dbp) {
    static std::multimap<uint256, CDiskBlockPos> mapBlocksUnknownParent;
    int nLoaded = 0;
    std::vector<unsigned char> buf;
    const unsigned char* magic = params.DiskMagic();
    uint64_t offset = 0;
    while (true) {
        unsigned char hdr[8];
        // resync on magic
        int c;
        int matched = 0;
        while (matched < 4 && (c = fgetc(fileIn)) != EOF) {
            offset++;
            if ((unsigned char)c == magic[matched]) matched++;
            else matched = ((unsigned char)c == magic[0]) ? 1 : 0;
        }
        if (matched < 4) break;
        if (fread(hdr + 4, 1, 4, fileIn) != 4) break;
        offset += 4;
        uint32_t nSize;
        memcpy(&nSize, hdr + 4, 4);
        if (nSize < 80 || nSize > 32 * 1000000) continue;
        buf.resize(nSize);
        const uint64_t blockPos = offset;
        if (fread(buf.data(), 1, nSize, fileIn) != nSize) break;
        offset += nSize;
        auto pblock = std::make_shared<CBlock>();
        if (!DecodeBlock(buf.data(), buf.size(), *pblock, pool.get())) continue; // transactions decoded in parallel
        const uint256 hash = pblock->GetHash(params.GetConsensus());
        CDiskBlockPos pos;
        if (dbp) {
            pos = *dbp;
            pos.nPos = (unsigned)blockPos;
        }
        {
            std::lock_guard<CCriticalSection> l(cs_main);
            if (hash != params.GetConsensus().hashGenesisBlock && !mapBlockIndex.count(pblock->hashPrevBlock)) {
                if (dbp) mapBlocksUnknownParent.insert(std::make_pair(pblock->hashPrevBlock, pos));
                continue;
            }
            CBlockIndex* existing = LookupBlockIndex(hash);
            if (existing && (existing->nStatus & BLOCK_HAVE_DATA)) continue;
            CValidationState state;
            if (AcceptBlock(pblock, state, nullptr, true, dbp ? &pos : nullptr, nullptr)) nLoaded++;
            if (state.IsError()) break;
        }
        CValidationState st;
        ActivateBestChain(st, pblock);
        // children that were waiting for this block
        std::deque<uint256> queue{hash};
        while (!queue.empty()) {
            const uint256 head = queue.front();
            queue.pop_front();
            auto range = mapBlocksUnknownParent.equal_range(head);
            while (range.first != range.second) {
                CDiskBlockPos childPos = range.first->second;
                auto child = std::make_shared<CBlock>();
                if (ReadBlockFromDisk(*child, childPos, params)) {
                    std::lock_guard<CCriticalSection> l(cs_main);
                    CValidationState dummy;
                    if (AcceptBlock(child, dummy, nullptr, true, &childPos, nullptr)) {
                        nLoaded++;
                        queue.push_back(child->GetHash(params.GetConsensus()));
                    }
                }
                range.first = mapBlocksUnknownParent.erase(range.first);
                CValidationState st2;
                ActivateBestChain(st2);
            }
        }
    }
    LogPrintf("Loaded %i blocks from external file\n", nLoaded);
    return nLoaded > 0;
}

bool Chainstate::Reindex() {
    {
        std::lock_guard<CCriticalSection> l(cs_main);
        pblocktree->WriteReindexing(true);
        fReindex = true;
    }
    std::string err;
    // genesis first (it lives in blk00000.dat at position 8)
    for (int nFile = 0;; nFile++) {
        CDiskBlockPos pos(nFile, 0);
        FILE* f = OpenBlockFile(pos, true);
        if (!f) break;
        LogPrintf("Reindexing block file blk%05u.dat...\n", (unsigned)nFile);
        LoadExternalBlockFile(f, &pos);
        fclose(f);
    }
    std::lock_guard<CCriticalSection> l(cs_main);
    pblocktree->WriteReindexing(false);
    fReindex = false;
    if (!InitBlockIndex(err)) return false;
    CValidationState state;
    ActivateBestChain(state);
    return true;
}

// ------------------------------------------------------------------ pruning
void Chainstate::PruneOneBlockFile(int fileNumber) {
    for (auto& kv : mapBlockIndex) {
        CBlockIndex* p = kv.second;
        if (p->nFile == fileNumber) {
            p->nStatus &= ~BLOCK_HAVE_DATA;
            p->nStatus &= ~BLOCK_HAVE_UNDO;
            p->nFile = 0;
            p->nDataPos = 0;
            p->nUndoPos = 0;
            setDirtyBlockIndex.insert(p);
            // blocks without data can no longer be candidates; keep them linkable
            auto range = mapBlocksUnlinked.equal_range(p->pprev);
            while (range.first != range.second) {
                if (range.first->second == p) range.first = mapBlocksUnlinked.erase(range.first);
                else ++range.first;
            }
        }
    }
    vinfoBlockFile[fileNumber] = CBlockFileInfo();
    setDirtyFileInfo.insert(fileNumber);
}

void Chainstate::UnlinkPrunedFiles(const std::set<int>& setFilesToPrune) {
    for (int f : setFilesToPrune) {
        CDiskBlockPos pos(f, 0);
        RemoveFile(GetBlockPosFilename(pos, "blk"));
        RemoveFile(GetBlockPosFilename(pos, "rev"));
        LogPrintf("Prune: deleted blk/rev (%05u)\n", (unsigned)f);
    }
}

void Chainstate::FindFilesToPruneManual(std::set<int>& setFilesToPrune, int nManualPruneHeight) {
    if (chainActive.Tip() == nullptr) return;
    const unsigned nLastBlockWeCanPrune = std::min((unsigned)nManualPruneHeight, chainActive.Tip()->nHeight - MIN_BLOCKS_TO_KEEP);
    for (int f = 0; f < nLastBlockFile; f++) {
        if (vinfoBlockFile[f].nSize == 0 || vinfoBlockFile[f].nHeightLast > nLastBlockWeCanPrune) continue;
        PruneOneBlockFile(f);
        setFilesToPrune.insert(f);
    }
}

void Chainstate::PruneBlockFilesManual(int nManualPruneHeight) {
    CValidationState state;
    FlushStateToDisk(state, FLUSH_STATE_NONE, nManualPruneHeight);
}

void Chainstate::FindFilesToPrune(std::set<int>& setFilesToPrune, uint64_t nPruneAfterHeight) {
    if (chainActive.Tip() == nullptr || opts.pruneTarget == 0) return;
    if ((uint64_t)chainActive.Tip()->nHeight <= nPruneAfterHeight) return;
    const unsigned nLastBlockWeCanPrune = chainActive.Tip()->nHeight - MIN_BLOCKS_TO_KEEP;
    uint64_t nCurrentUsage = CalculateCurrentUsage();
    const uint64_t nBuffer = FileSizes().blockChunk + FileSizes().undoChunk;
    if (nCurrentUsage + nBuffer < opts.pruneTarget) return;
    for (int f = 0; f < nLastBlockFile; f++) {
        const uint64_t nBytesToPrune = vinfoBlockFile[f].nSize + vinfoBlockFile[f].nUndoSize;
        if (vinfoBlockFile[f].nSize == 0) continue;
        if (nCurrentUsage + nBuffer < opts.pruneTarget) break;
        if (vinfoBlockFile[f].nHeightLast > nLastBlockWeCanPrune) continue;
        PruneOneBlockFile(f);
        setFilesToPrune.insert(f);
        nCurrentUsage -= nBytesToPrune;
    }
}

} // namespace bcp
