#include "net/net_processing.h"
#include "consensus/merkleblock.h"
#include "consensus/tx_verify.h"
#include "net/blockencodings.h"
#include "node/policy.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "node/ui_interface.h"
#include "node/warnings.h"
#include "util/strencodings.h"

#include <algorithm>

namespace bcp {

static PeerLogicValidation* g_peerlogic = nullptr;
PeerLogicValidation* GetPeerLogic() { return g_peerlogic; }

namespace {

// Bounded string read (reference serialize.h LIMITED_STRING).
template <typename S> void ReadLimitedString(S& s, std::string& out, size_t limit) {
    const uint64_t n = ReadCompactSize(s);
    if (n > limit) throw ser_error("String length limit exceeded");
    out.resize(n);
    if (n) s.read(&out[0], n);
}

// A "headers" payload is a vector of blocks with no transactions (each entry carries a
// zero tx count), reference net_processing.cpp getheaders reply.
std::vector<CBlock> HeadersForWire(const std::vector<CBlockHeader>& v) {
    std::vector<CBlock> out;
    out.reserve(v.size());
    for (const CBlockHeader& h : v) out.emplace_back(h);
    return out;
}

struct QueuedBlock {
    uint256 hash;
    const CBlockIndex* pindex;
    bool fValidatedHeaders;
    std::unique_ptr<PartiallyDownloadedBlock> partialBlock;
};

struct CNodeState {
    CAddress address;
    std::string name;
    bool fCurrentlyConnected = false;
    int nMisbehavior = 0;
    bool fShouldBan = false;
    const CBlockIndex* pindexBestKnownBlock = nullptr;
    uint256 hashLastUnknownBlock;
    const CBlockIndex* pindexLastCommonBlock = nullptr;
    const CBlockIndex* pindexBestHeaderSent = nullptr;
    int nUnconnectingHeaders = 0;
    bool fSyncStarted = false;
    int64_t nHeadersSyncTimeout = 0;
    int64_t nStallingSince = 0;
    std::list<QueuedBlock> vBlocksInFlight;
    int64_t nDownloadingSince = 0;
    int nBlocksInFlight = 0;
    int nBlocksInFlightValidHeaders = 0;
    bool fPreferredDownload = false;
    bool fPreferHeaders = false;
    bool fPreferHeaderAndIDs = false;
    bool fProvidesHeaderAndIDs = false;
    bool fSupportsDesiredCmpctVersion = false;
    struct Reject {
        unsigned char code;
        std::string reason;
        uint256 hash;
    };
    std::vector<Reject> rejects;
};

struct COrphanTx {
    CTransactionRef tx;
    NodeId fromPeer;
    int64_t nTimeExpire;
};

} // namespace

struct PeerLogicValidation::Impl {
    CConnman* connman;
    Chainstate* cs;
    CTxMemPool* pool;
    std::map<NodeId, CNodeState> mapNodeState;
    std::map<uint256, std::pair<NodeId, std::list<QueuedBlock>::iterator>> mapBlocksInFlight;
    std::map<uint256, std::pair<NodeId, bool>> mapBlockSource; // block -> (peer, punish)
    std::list<NodeId> lNodesAnnouncingHeaderAndIDs;
    int nSyncStarted = 0;
    int nPreferredDownload = 0;
    int nPeersWithValidatedDownloads = 0;
    // orphans
    std::mutex cs_orphans;
    std::map<uint256, COrphanTx> mapOrphanTransactions;
    std::map<COutPoint, std::set<uint256>> mapOrphanTransactionsByPrev;
    int64_t nNextOrphanSweep = 0;
    // recently rejected / relay cache
    CRollingBloomFilter recentRejects{120000, 0.000001};
    uint256 hashRecentRejectsChainTip;
    std::map<uint256, CTransactionRef> mapRelay;
    std::deque<std::pair<int64_t, uint256>> vRelayExpiration;
    // extra txn for compact block reconstruction
    std::vector<std::pair<uint256, CTransactionRef>> vExtraTxnForCompact;
    size_t vExtraTxnForCompactIt = 0;
    // most recent block for fast cmpctblock relay
    std::mutex cs_most_recent;
    std::shared_ptr<const CBlock> most_recent_block;
    std::shared_ptr<const CBlockHeaderAndShortTxIDs> most_recent_compact_block;
    uint256 most_recent_block_hash;
    int64_t nTimeBestReceived = 0;
    FastRandomContext rng;

    CCriticalSection& csMain() RETURN_CAPABILITY(cs->cs()) { return cs->cs(); }
    CNodeState* State(NodeId id) {
        auto it = mapNodeState.find(id);
        return it == mapNodeState.end() ? nullptr : &it->second;
    }
    void Push(CNode* p, CSerializedNetMsg&& m) { connman->PushMessage(p, std::move(m)); }

    void MisbehavingLocked(NodeId id, int howmuch, const std::string& reason) {
        if (howmuch == 0) return;
        CNodeState* st = State(id);
        if (!st) return;
        st->nMisbehavior += howmuch;
        const int banscore = (int)gArgs.GetArg("-banscore", DEFAULT_BANSCORE_THRESHOLD);
        if (st->nMisbehavior >= banscore && st->nMisbehavior - howmuch < banscore) {
            LogPrintf("%s: %s peer=%d (%d -> %d) reason: %s BAN THRESHOLD EXCEEDED\n", __func__, st->name.c_str(),
                      (int)id, st->nMisbehavior - howmuch, st->nMisbehavior, reason.c_str());
            st->fShouldBan = true;
        } else {
            LogPrintf("%s: %s peer=%d (%d -> %d) reason: %s\n", __func__, st->name.c_str(), (int)id,
                      st->nMisbehavior - howmuch, st->nMisbehavior, reason.c_str());
        }
    }

    void Misbehaving(NodeId id, int howmuch, const std::string& reason = "") {
        std::lock_guard<CCriticalSection> l(csMain());
        MisbehavingLocked(id, howmuch, reason);
    }

    void UpdatePreferredDownload(CNode* p, CNodeState* st) {
        nPreferredDownload -= st->fPreferredDownload;
        st->fPreferredDownload = (!p->fInbound || p->fWhitelisted) && !p->fOneShot && !p->fClient;
        nPreferredDownload += st->fPreferredDownload;
    }

    bool MarkBlockAsReceived(const uint256& hash) {
        auto it = mapBlocksInFlight.find(hash);
        if (it == mapBlocksInFlight.end()) return false;
        CNodeState* st = State(it->second.first);
        if (st) {
            st->nBlocksInFlightValidHeaders -= it->second.second->fValidatedHeaders;
            if (st->nBlocksInFlightValidHeaders == 0 && it->second.second->fValidatedHeaders)
                nPeersWithValidatedDownloads--;
            if (st->vBlocksInFlight.begin() == it->second.second) st->nDownloadingSince = std::max(st->nDownloadingSince, GetTimeMicros());
            st->vBlocksInFlight.erase(it->second.second);
            st->nBlocksInFlight--;
            st->nStallingSince = 0;
        }
        mapBlocksInFlight.erase(it);
        return true;
    }

    bool MarkBlockAsInFlight(NodeId id, const uint256& hash, const CBlockIndex* pindex,
                             std::list<QueuedBlock>::iterator** pit = nullptr) {
        CNodeState* st = State(id);
        if (!st) return false;
        auto it = mapBlocksInFlight.find(hash);
        if (it != mapBlocksInFlight.end() && it->second.first == id) {
            if (pit) *pit = &it->second.second;
            return false;
        }
        MarkBlockAsReceived(hash);
        QueuedBlock qb;
        qb.hash = hash;
        qb.pindex = pindex;
        qb.fValidatedHeaders = pindex != nullptr;
        if (pit) qb.partialBlock.reset(new PartiallyDownloadedBlock(pool));
        auto qit = st->vBlocksInFlight.insert(st->vBlocksInFlight.end(), std::move(qb));
        st->nBlocksInFlight++;
        st->nBlocksInFlightValidHeaders += qit->fValidatedHeaders;
        if (st->nBlocksInFlight == 1) st->nDownloadingSince = GetTimeMicros();
        if (st->nBlocksInFlightValidHeaders == 1 && pindex) nPeersWithValidatedDownloads++;
        auto& slot = mapBlocksInFlight[hash];
        slot = {id, qit};
        if (pit) *pit = &slot.second;
        return true;
    }

    void ProcessBlockAvailability(NodeId id) {
        CNodeState* st = State(id);
        if (!st->hashLastUnknownBlock.IsNull()) {
            const CBlockIndex* pi = cs->LookupBlockIndex(st->hashLastUnknownBlock);
            if (pi && pi->nChainWork > 0) {
                if (!st->pindexBestKnownBlock || pi->nChainWork >= st->pindexBestKnownBlock->nChainWork)
                    st->pindexBestKnownBlock = pi;
                st->hashLastUnknownBlock.SetNull();
            }
        }
    }

    void UpdateBlockAvailability(NodeId id, const uint256& hash) {
        CNodeState* st = State(id);
        if (!st) return;
        ProcessBlockAvailability(id);
        const CBlockIndex* pi = cs->LookupBlockIndex(hash);
        if (pi && pi->nChainWork > 0) {
            if (!st->pindexBestKnownBlock || pi->nChainWork >= st->pindexBestKnownBlock->nChainWork)
                st->pindexBestKnownBlock = pi;
        } else {
            st->hashLastUnknownBlock = hash;
        }
    }

    bool CanDirectFetch() EXCLUSIVE_LOCKS_REQUIRED(csMain()) {
        return cs->Tip()->GetBlockTime() > GetAdjustedTime() - cs->Params().GetConsensus().nPowTargetSpacing * 20;
    }

    bool PeerHasHeader(CNodeState* st, const CBlockIndex* pindex) {
        if (st->pindexBestKnownBlock && pindex == st->pindexBestKnownBlock->GetAncestor(pindex->nHeight)) return true;
        if (st->pindexBestHeaderSent && pindex == st->pindexBestHeaderSent->GetAncestor(pindex->nHeight)) return true;
        return false;
    }

    void FindNextBlocksToDownload(NodeId id, unsigned count, std::vector<const CBlockIndex*>& vBlocks, NodeId& nodeStaller)
        EXCLUSIVE_LOCKS_REQUIRED(csMain()) {
        if (count == 0) return;
        vBlocks.reserve(vBlocks.size() + count);
        CNodeState* st = State(id);
        ProcessBlockAvailability(id);
        if (!st->pindexBestKnownBlock || st->pindexBestKnownBlock->nChainWork < cs->Tip()->nChainWork) return;
        if (!st->pindexLastCommonBlock) {
            st->pindexLastCommonBlock =
                cs->ActiveChain()[std::min(st->pindexBestKnownBlock->nHeight, cs->Height())];
        }
        st->pindexLastCommonBlock = LastCommonAncestor(st->pindexLastCommonBlock, st->pindexBestKnownBlock);
        if (st->pindexLastCommonBlock == st->pindexBestKnownBlock) return;
        std::vector<const CBlockIndex*> vToFetch;
        const CBlockIndex* pindexWalk = st->pindexLastCommonBlock;
        const int nWindowEnd = st->pindexLastCommonBlock->nHeight + BLOCK_DOWNLOAD_WINDOW;
        const int nMaxHeight = std::min<int>(st->pindexBestKnownBlock->nHeight, nWindowEnd + 1);
        NodeId waitingfor = -1;
        while (pindexWalk->nHeight < nMaxHeight) {
            const int nToFetch = std::min(nMaxHeight - pindexWalk->nHeight, std::max<int>(count - vBlocks.size(), 128));
            vToFetch.resize(nToFetch);
            pindexWalk = st->pindexBestKnownBlock->GetAncestor(pindexWalk->nHeight + nToFetch);
            vToFetch[nToFetch - 1] = pindexWalk;
            for (int i = nToFetch - 1; i > 0; i--) vToFetch[i - 1] = vToFetch[i]->pprev;
            for (const CBlockIndex* pi : vToFetch) {
                if (!pi->IsValid(BLOCK_VALID_TREE)) return; // invalid chain
                if (pi->nStatus & BLOCK_HAVE_DATA || cs->ActiveChain().Contains(pi)) {
                    if (pi->nChainTx) st->pindexLastCommonBlock = pi;
                } else if (mapBlocksInFlight.count(pi->GetBlockHash()) == 0) {
                    if (pi->nHeight > nWindowEnd) {
                        if (vBlocks.empty() && waitingfor != id) nodeStaller = waitingfor;
                        return;
                    }
                    vBlocks.push_back(pi);
                    if (vBlocks.size() == count) return;
                } else if (waitingfor == -1) {
                    waitingfor = mapBlocksInFlight[pi->GetBlockHash()].first;
                }
            }
        }
    }

    // ---- orphans (reference net_processing.cpp AddOrphanTx/EraseOrphanTx/LimitOrphanTxSize)
    bool AddOrphanTx(const CTransactionRef& tx, NodeId peer) {
        std::lock_guard<std::mutex> l(cs_orphans);
        const uint256 h = tx->GetHash();
        if (mapOrphanTransactions.count(h)) return false;
        const size_t sz = GetSerializeSize(*tx);
        if (sz >= 100000) {
            LogPrint(BCLog::MEMPOOL, "ignoring large orphan tx (size: %zu, hash: %s)\n", sz, h.ToString().c_str());
            return false;
        }
        mapOrphanTransactions[h] = {tx, peer, GetTime() + ORPHAN_TX_EXPIRE_TIME};
        for (const CTxIn& in : tx->vin) mapOrphanTransactionsByPrev[in.prevout].insert(h);
        AddToCompactExtraTransactions(tx);
        LogPrint(BCLog::MEMPOOL, "stored orphan tx %s (mapsz %zu outsz %zu)\n", h.ToString().c_str(),
                 mapOrphanTransactions.size(), mapOrphanTransactionsByPrev.size());
        return true;
    }
    int EraseOrphanTxLocked(const uint256& h) {
        auto it = mapOrphanTransactions.find(h);
        if (it == mapOrphanTransactions.end()) return 0;
        for (const CTxIn& in : it->second.tx->vin) {
            auto pit = mapOrphanTransactionsByPrev.find(in.prevout);
            if (pit == mapOrphanTransactionsByPrev.end()) continue;
            pit->second.erase(h);
            if (pit->second.empty()) mapOrphanTransactionsByPrev.erase(pit);
        }
        mapOrphanTransactions.erase(it);
        return 1;
    }
    void EraseOrphansFor(NodeId peer) {
        std::lock_guard<std::mutex> l(cs_orphans);
        int n = 0;
        for (auto it = mapOrphanTransactions.begin(); it != mapOrphanTransactions.end();) {
            auto cur = it++;
            if (cur->second.fromPeer == peer) n += EraseOrphanTxLocked(cur->first);
        }
        if (n) LogPrint(BCLog::MEMPOOL, "Erased %d orphan tx from peer=%d\n", n, (int)peer);
    }
    unsigned LimitOrphanTxSize(unsigned nMax) {
        std::lock_guard<std::mutex> l(cs_orphans);
        unsigned nEvicted = 0;
        const int64_t now = GetTime();
        if (nNextOrphanSweep <= now) {
            int64_t nMinExpTime = now + ORPHAN_TX_EXPIRE_TIME - ORPHAN_TX_EXPIRE_INTERVAL;
            for (auto it = mapOrphanTransactions.begin(); it != mapOrphanTransactions.end();) {
                auto cur = it++;
                if (cur->second.nTimeExpire <= now)
                    EraseOrphanTxLocked(cur->first);
                else
                    nMinExpTime = std::min(cur->second.nTimeExpire, nMinExpTime);
            }
            nNextOrphanSweep = nMinExpTime + ORPHAN_TX_EXPIRE_INTERVAL;
        }
        while (mapOrphanTransactions.size() > nMax) {
            auto it = mapOrphanTransactions.lower_bound(GetRandHash());
            if (it == mapOrphanTransactions.end()) it = mapOrphanTransactions.begin();
            EraseOrphanTxLocked(it->first);
            nEvicted++;
        }
        return nEvicted;
    }
    void AddToCompactExtraTransactions(const CTransactionRef& tx) {
        const size_t max = (size_t)gArgs.GetArg("-blockreconstructionextratxn", (int64_t)100);
        if (max == 0) return;
        if (vExtraTxnForCompact.empty()) vExtraTxnForCompact.resize(max);
        vExtraTxnForCompact[vExtraTxnForCompactIt] = {tx->GetHash(), tx};
        vExtraTxnForCompactIt = (vExtraTxnForCompactIt + 1) % max;
    }

    bool AlreadyHave(const CInv& inv) EXCLUSIVE_LOCKS_REQUIRED(csMain()) {
        switch (inv.type) {
        case MSG_TX: {
            if (cs->Tip()->GetBlockHash() != hashRecentRejectsChainTip) {
                hashRecentRejectsChainTip = cs->Tip()->GetBlockHash();
                recentRejects.reset();
            }
            if (recentRejects.contains(inv.hash)) return true;
            if (pool->exists(inv.hash)) return true;
            {
                std::lock_guard<std::mutex> l(cs_orphans);
                if (mapOrphanTransactions.count(inv.hash)) return true;
            }
            const CCoinsViewCache& coins = cs->CoinsTip();
            return coins.HaveCoinInCache(COutPoint(inv.hash, 0)) || coins.HaveCoinInCache(COutPoint(inv.hash, 1));
        }
        case MSG_BLOCK: return cs->LookupBlockIndex(inv.hash) != nullptr;
        }
        return true;
    }

    void RelayAddress(const CAddress& addr, bool fReachable) {
        // relay to 1 or 2 deterministic-random peers per 24h window
        const unsigned nRelayNodes = fReachable ? 2 : 1;
        const uint64_t hashAddr = addr.GetHash();
        const CSipHasher hasher =
            connman->GetDeterministicRandomizer(0x9b5b5c8c1f4e3a37ULL).Write(hashAddr << 32).Write((GetTime() + hashAddr) / (24 * 60 * 60));
        std::vector<std::pair<uint64_t, CNode*>> best;
        connman->ForEachNode([&](CNode* p) {
            if (p->nVersion < CADDR_TIME_VERSION) return;
            const uint64_t key = CSipHasher(hasher).Write(p->GetId()).Finalize();
            best.push_back({key, p});
        });
        std::sort(best.begin(), best.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        for (size_t i = 0; i < nRelayNodes && i < best.size(); i++) best[i].second->PushAddress(addr, rng);
    }

    void RelayTransaction(const CTransaction& tx) {
        const uint256 h = tx.GetHash();
        {
            const int64_t now = GetTime();
            while (!vRelayExpiration.empty() && vRelayExpiration.front().first < now) {
                mapRelay.erase(vRelayExpiration.front().second);
                vRelayExpiration.pop_front();
            }
            if (mapRelay.emplace(h, std::make_shared<const CTransaction>(tx)).second)
                vRelayExpiration.push_back({now + 15 * 60, h});
        }
        connman->RelayTransaction(tx);
    }

    // ---- message handlers
    void ProcessGetData(CNode* pfrom, std::deque<CInv>& vRecvGetData, std::atomic<bool>& interrupt);
    bool ProcessMessage(CNode* pfrom, const std::string& strCommand, DataStream& vRecv, int64_t nTimeReceived,
                        std::atomic<bool>& interrupt);
    bool ProcessHeadersMessage(CNode* pfrom, const std::vector<CBlockHeader>& headers, bool punishDuplicateInvalid);
    void ProcessOrphans(std::set<uint256>& work);
    bool SendRejectsAndCheckIfBanned(CNode* pnode);
    void PushNodeVersion(CNode* pnode, int64_t nTime);
    std::map<NodeId, std::deque<CInv>> mapGetData;
};

PeerLogicValidation::PeerLogicValidation(CConnman* connman, Chainstate* chainstate, CTxMemPool* mempool)
    : impl(new Impl()) {
    impl->connman = connman;
    impl->cs = chainstate;
    impl->pool = mempool;
    g_peerlogic = this;
}

PeerLogicValidation::~PeerLogicValidation() {
    if (g_peerlogic == this) g_peerlogic = nullptr;
}

void PeerLogicValidation::Impl::PushNodeVersion(CNode* pnode, int64_t nTime) {
    const uint64_t nLocalNodeServices = pnode->GetLocalServices();
    const uint64_t nonce = pnode->GetLocalNonce();
    const int nNodeStartingHeight = pnode->GetMyStartingHeight();
    const CAddress addrYou = pnode->addr.IsRoutable() ? pnode->addr : CAddress(CService(), pnode->addr.nServices);
    const CAddress addrMe(CService(), nLocalNodeServices);
    const bool fRelay = !gArgs.GetBoolArg("-blocksonly", false);
    Push(pnode, CNetMsgMaker(INIT_PROTO_VERSION)
                    .Make(NetMsgType::VERSION, PROTOCOL_VERSION, nLocalNodeServices, nTime, addrYou, addrMe, nonce,
                          UserAgent(cs->MaxBlockSize()), nNodeStartingHeight, fRelay));
    LogPrint(BCLog::NET, "send version message: version %d, blocks=%d, us=%s, peer=%d\n", PROTOCOL_VERSION,
             nNodeStartingHeight, addrMe.ToString().c_str(), (int)pnode->GetId());
}

void PeerLogicValidation::InitializeNode(CNode* pnode) {
    {
        std::lock_guard<CCriticalSection> l(impl->csMain());
        CNodeState& st = impl->mapNodeState[pnode->GetId()];
        st.address = pnode->addr;
        st.name = pnode->GetAddrName();
    }
    if (!pnode->fInbound) impl->PushNodeVersion(pnode, GetAdjustedTime());
}

void PeerLogicValidation::FinalizeNode(NodeId id, bool& fUpdateConnectionTime) {
    fUpdateConnectionTime = false;
    std::lock_guard<CCriticalSection> l(impl->csMain());
    CNodeState* st = impl->State(id);
    if (!st) return;
    if (st->fSyncStarted) impl->nSyncStarted--;
    if (st->nMisbehavior == 0 && st->fCurrentlyConnected) fUpdateConnectionTime = true;
    for (const QueuedBlock& qb : st->vBlocksInFlight) impl->mapBlocksInFlight.erase(qb.hash);
    impl->EraseOrphansFor(id);
    impl->nPreferredDownload -= st->fPreferredDownload;
    impl->nPeersWithValidatedDownloads -= (st->nBlocksInFlightValidHeaders != 0);
    impl->mapNodeState.erase(id);
    impl->mapGetData.erase(id);
    impl->lNodesAnnouncingHeaderAndIDs.remove(id);
    if (impl->mapNodeState.empty()) {
        impl->nPreferredDownload = 0;
        impl->nPeersWithValidatedDownloads = 0;
    }
    LogPrint(BCLog::NET, "Cleared nodestate for peer=%d\n", (int)id);
}

bool PeerLogicValidation::GetNodeStateStats(NodeId id, CNodeStateStats& stats) {
    std::lock_guard<CCriticalSection> l(impl->csMain());
    CNodeState* st = impl->State(id);
    if (!st) return false;
    stats.nMisbehavior = st->nMisbehavior;
    stats.nSyncHeight = st->pindexBestKnownBlock ? st->pindexBestKnownBlock->nHeight : -1;
    stats.nCommonHeight = st->pindexLastCommonBlock ? st->pindexLastCommonBlock->nHeight : -1;
    for (const QueuedBlock& qb : st->vBlocksInFlight)
        if (qb.pindex) stats.vHeightInFlight.push_back(qb.pindex->nHeight);
    return true;
}

void PeerLogicValidation::Misbehaving(NodeId id, int howmuch, const std::string& reason) {
    std::lock_guard<CCriticalSection> l(impl->csMain());
    impl->MisbehavingLocked(id, howmuch, reason);
}

bool PeerLogicValidation::AddOrphanTx(const CTransactionRef& tx, NodeId peer) { return impl->AddOrphanTx(tx, peer); }
void PeerLogicValidation::EraseOrphansFor(NodeId peer) { impl->EraseOrphansFor(peer); }
unsigned PeerLogicValidation::LimitOrphanTxSize(unsigned nMaxOrphans) { return impl->LimitOrphanTxSize(nMaxOrphans); }

size_t PeerLogicValidation::OrphanCount() {
    std::lock_guard<std::mutex> l(impl->cs_orphans);
    return impl->mapOrphanTransactions.size();
}

void PeerLogicValidation::RelayTransaction(const CTransaction& tx) {
    std::lock_guard<CCriticalSection> l(impl->csMain());
    impl->RelayTransaction(tx);
}

// ------------------------------------------------------------------ validation callbacks
void PeerLogicValidation::UpdatedBlockTip(const CBlockIndex* pindexNew, const CBlockIndex* pindexFork,
                                          bool fInitialDownload) {
    const int nNewHeight = pindexNew->nHeight;
    impl->connman->SetBestHeight(nNewHeight);
    if (!fInitialDownload) {
        std::vector<uint256> vHashes;
        const CBlockIndex* pi = pindexNew;
        while (pi && pi != pindexFork) {
            vHashes.push_back(pi->GetBlockHash());
            pi = pi->pprev;
            if (vHashes.size() == MAX_BLOCKS_TO_ANNOUNCE) break;
        }
        impl->connman->ForEachNode([&](CNode* p) {
            if (nNewHeight > (p->nStartingHeight != -1 ? p->nStartingHeight - 2000 : 0))
                for (auto it = vHashes.rbegin(); it != vHashes.rend(); ++it) p->PushBlockHash(*it);
        });
        impl->connman->WakeMessageHandler();
    }
    impl->nTimeBestReceived = GetTime();
}

void PeerLogicValidation::BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex*,
                                         const std::vector<CTransactionRef>&) {
    std::lock_guard<std::mutex> l(impl->cs_orphans);
    std::vector<uint256> vOrphanErase;
    for (const CTransactionRef& tx : block->vtx) {
        for (const CTxIn& in : tx->vin) {
            auto it = impl->mapOrphanTransactionsByPrev.find(in.prevout);
            if (it == impl->mapOrphanTransactionsByPrev.end()) continue;
            for (const uint256& h : it->second) vOrphanErase.push_back(h);
        }
    }
    for (const uint256& h : vOrphanErase) impl->EraseOrphanTxLocked(h);
}

void PeerLogicValidation::NewPoWValidBlock(const CBlockIndex* pindex, const std::shared_ptr<const CBlock>& pblock) {
    auto pcmpct = std::make_shared<const CBlockHeaderAndShortTxIDs>(*pblock, impl->rng.rand64());
    std::lock_guard<CCriticalSection> l(impl->csMain());
    static int nHighestFastAnnounce = 0;
    if (pindex->nHeight <= nHighestFastAnnounce) return;
    nHighestFastAnnounce = pindex->nHeight;
    const uint256 hash = pblock->GetHash();
    {
        std::lock_guard<std::mutex> lr(impl->cs_most_recent);
        impl->most_recent_block_hash = hash;
        impl->most_recent_block = pblock;
        impl->most_recent_compact_block = pcmpct;
    }
    impl->connman->ForEachNode([&](CNode* p) {
        if (p->nVersion < INVALID_CB_NO_BAN_VERSION || p->fDisconnect) return;
        CNodeState* st = impl->State(p->GetId());
        if (!st) return;
        if (st->fPreferHeaderAndIDs && !impl->PeerHasHeader(st, pindex) && impl->PeerHasHeader(st, pindex->pprev)) {
            LogPrint(BCLog::NET, "%s sending header-and-ids %s to peer=%d\n", "PeerLogicValidation::NewPoWValidBlock",
                     hash.ToString().c_str(), (int)p->GetId());
            impl->Push(p, CNetMsgMaker(p->GetSendVersion()).Make(NetMsgType::CMPCTBLOCK, *pcmpct));
            st->pindexBestHeaderSent = pindex;
        }
    });
}

void PeerLogicValidation::BlockChecked(const CBlock& block, const CValidationState& state) {
    std::lock_guard<CCriticalSection> l(impl->csMain());
    const uint256 hash = block.GetHash();
    auto it = impl->mapBlockSource.find(hash);
    int nDoS = 0;
    if (state.IsInvalid(nDoS)) {
        if (it != impl->mapBlockSource.end() && impl->State(it->second.first)) {
            CNodeState* st = impl->State(it->second.first);
            st->rejects.push_back({(unsigned char)state.GetRejectCode(), state.GetRejectReason().substr(0, 111), hash});
            if (nDoS > 0 && it->second.second) impl->MisbehavingLocked(it->second.first, nDoS, state.GetRejectReason());
        }
    } else if (state.IsValid() && !impl->cs->IsInitialBlockDownload() &&
               impl->mapBlocksInFlight.count(hash) == impl->mapBlocksInFlight.size()) {
        // block relayed over compact blocks by a peer: keep it as a high-bandwidth announcer
        if (it != impl->mapBlockSource.end()) {
            const NodeId nodeid = it->second.first;
            auto& lst = impl->lNodesAnnouncingHeaderAndIDs;
            CNodeState* st = impl->State(nodeid);
            if (st && st->fSupportsDesiredCmpctVersion &&
                std::find(lst.begin(), lst.end(), nodeid) == lst.end()) {
                impl->connman->ForNode(nodeid, [&](CNode* pfrom) {
                    bool fAnnounceUsingCMPCTBLOCK = false;
                    uint64_t nCMPCTBLOCKVersion = 1;
                    if (lst.size() >= 3) {
                        impl->connman->ForNode(lst.front(), [&](CNode* old) {
                            bool f = false;
                            impl->Push(old, CNetMsgMaker(old->GetSendVersion())
                                                .Make(NetMsgType::SENDCMPCT, f, nCMPCTBLOCKVersion));
                            return true;
                        });
                        lst.pop_front();
                    }
                    fAnnounceUsingCMPCTBLOCK = true;
                    impl->Push(pfrom, CNetMsgMaker(pfrom->GetSendVersion())
                                          .Make(NetMsgType::SENDCMPCT, fAnnounceUsingCMPCTBLOCK, nCMPCTBLOCKVersion));
                    lst.push_back(pfrom->GetId());
                    return true;
                });
            }
        }
    }
    if (it != impl->mapBlockSource.end()) impl->mapBlockSource.erase(it);
}

void PeerLogicValidation::TransactionAddedToMempool(const CTransactionRef&) {}

// ------------------------------------------------------------------ getdata
void PeerLogicValidation::Impl::ProcessGetData(CNode* pfrom, std::deque<CInv>& vRecvGetData,
                                               std::atomic<bool>& interrupt) {
    std::vector<CInv> vNotFound;
    const CNetMsgMaker msgMaker(pfrom->GetSendVersion());
    const int legacyFlag = pfrom->IsLegacyBlockHeader(pfrom->GetSendVersion()) ? SERIALIZE_BLOCK_LEGACY : 0;
    std::lock_guard<CCriticalSection> l(csMain());
    auto it = vRecvGetData.begin();
    while (it != vRecvGetData.end()) {
        if (pfrom->fPauseSend) break;
        const CInv& inv = *it;
        if (interrupt) return;
        it++;
        if (inv.type == MSG_BLOCK || inv.type == MSG_FILTERED_BLOCK || inv.type == MSG_CMPCT_BLOCK) {
            bool send = false;
            const CBlockIndex* pi = cs->LookupBlockIndex(inv.hash);
            if (pi) {
                if (pi->nChainTx && !pi->IsValid(BLOCK_VALID_SCRIPTS) && pi->IsValid(BLOCK_VALID_TREE)) {
                    // The block and all its parents are here but not yet validated: this node may be
                    // between AcceptBlock and ActivateBestChain of that block (its compact-block
                    // announcement, NewPoWValidBlock, goes out first, and a peer asks for it right
                    // away). Connect it now so the relay check below sees it; otherwise the request
                    // is dropped and the peer waits for the block until its download times out
                    // (reference net_processing.cpp:1164-1180).
                    std::shared_ptr<const CBlock> recent;
                    {
                        std::lock_guard<std::mutex> lr(cs_most_recent);
                        recent = most_recent_block;
                    }
                    CValidationState dummy;
                    cs->ActivateBestChain(dummy, recent);
                }
                if (cs->ActiveChain().Contains(pi)) {
                    send = true;
                } else {
                    // anti-fingerprinting: only serve side-chain blocks that are valid and recent
                    static const int nOneMonth = 30 * 24 * 60 * 60;
                    send = pi->IsValid(BLOCK_VALID_SCRIPTS) && cs->BestHeader() &&
                           cs->BestHeader()->GetBlockTime() - pi->GetBlockTime() < nOneMonth;
                    if (!send)
                        LogPrintf("%s: ignoring request from peer=%d for old block that isn't in the main chain\n",
                                  __func__, (int)pfrom->GetId());
                }
            }
            // historical block serving limit
            static const int nOneWeek = 7 * 24 * 60 * 60;
            if (send && connman->OutboundTargetReached(true) && cs->BestHeader() &&
                (cs->BestHeader()->GetBlockTime() - pi->GetBlockTime() > nOneWeek) && !pfrom->fWhitelisted) {
                LogPrint(BCLog::NET, "historical block serving limit reached, disconnect peer=%d\n", (int)pfrom->GetId());
                pfrom->fDisconnect = true;
                send = false;
            }
            if (send && (pi->nStatus & BLOCK_HAVE_DATA)) {
                std::shared_ptr<const CBlock> pblock;
                {
                    std::lock_guard<std::mutex> lr(cs_most_recent);
                    if (most_recent_block && most_recent_block_hash == pi->GetBlockHash()) pblock = most_recent_block;
                }
                if (!pblock) {
                    auto b = std::make_shared<CBlock>();
                    if (!cs->ReadBlock(*b, pi, false)) {
                        LogPrintf("cannot load block from disk\n");
                        continue;
                    }
                    pblock = b;
                }
                if (inv.type == MSG_BLOCK) {
                    Push(pfrom, msgMaker.Make(legacyFlag, NetMsgType::BLOCK, *pblock));
                } else if (inv.type == MSG_FILTERED_BLOCK) {
                    bool sendMerkle = false;
                    CMerkleBlock merkleBlock;
                    {
                        std::lock_guard<std::mutex> lf(pfrom->cs_filter);
                        if (pfrom->pfilter) {
                            sendMerkle = true;
                            merkleBlock = CMerkleBlock(*pblock, *pfrom->pfilter);
                        }
                    }
                    if (sendMerkle) {
                        Push(pfrom, msgMaker.Make(legacyFlag, NetMsgType::MERKLEBLOCK, merkleBlock));
                        for (const auto& pair : merkleBlock.vMatchedTxn)
                            Push(pfrom, msgMaker.Make(NetMsgType::TX, *pblock->vtx[pair.first]));
                    }
                } else if (inv.type == MSG_CMPCT_BLOCK) {
                    if (CanDirectFetch() && pi->nHeight >= cs->Height() - MAX_CMPCTBLOCK_DEPTH) {
                        CBlockHeaderAndShortTxIDs cmpct(*pblock, rng.rand64());
                        Push(pfrom, msgMaker.Make(legacyFlag, NetMsgType::CMPCTBLOCK, cmpct));
                    } else {
                        Push(pfrom, msgMaker.Make(legacyFlag, NetMsgType::BLOCK, *pblock));
                    }
                }
                // continuation of getblocks: announce the tip so the peer asks for more
                if (inv.hash == pfrom->hashContinue) {
                    std::vector<CInv> vInv{CInv(MSG_BLOCK, cs->Tip()->GetBlockHash())};
                    Push(pfrom, msgMaker.Make(NetMsgType::INV, vInv));
                    pfrom->hashContinue.SetNull();
                }
            }
        } else if (inv.type == MSG_TX) {
            CTransactionRef tx;
            auto mr = mapRelay.find(inv.hash);
            if (mr != mapRelay.end()) {
                tx = mr->second;
            } else if (pfrom->timeLastMempoolReq) {
                TxMempoolInfo info = pool->info(inv.hash);
                if (info.tx && info.nTime <= pfrom->timeLastMempoolReq) tx = info.tx;
            }
            if (!tx) tx = pool->get(inv.hash);
            if (tx)
                Push(pfrom, msgMaker.Make(NetMsgType::TX, *tx));
            else
                vNotFound.push_back(inv);
        } else {
            vNotFound.push_back(inv);
        }
        // one block per call so other peers get serviced
        if (inv.type == MSG_BLOCK || inv.type == MSG_FILTERED_BLOCK || inv.type == MSG_CMPCT_BLOCK) break;
    }
    vRecvGetData.erase(vRecvGetData.begin(), it);
    if (!vNotFound.empty()) Push(pfrom, msgMaker.Make(NetMsgType::NOTFOUND, vNotFound));
}

// ------------------------------------------------------------------ headers
bool PeerLogicValidation::Impl::ProcessHeadersMessage(CNode* pfrom, const std::vector<CBlockHeader>& headers,
                                                      bool punishDuplicateInvalid) {
    const CNetMsgMaker msgMaker(pfrom->GetSendVersion());
    const size_t nCount = headers.size();
    if (nCount == 0) return true;
    bool received_new_header = false;
    const CBlockIndex* pindexLast = nullptr;
    {
        std::lock_guard<CCriticalSection> l(csMain());
        CNodeState* st = State(pfrom->GetId());
        // unconnecting headers: ask for the gap, punish repeated offenders
        if (!cs->LookupBlockIndex(headers[0].hashPrevBlock) && nCount < MAX_BLOCKS_TO_ANNOUNCE) {
            st->nUnconnectingHeaders++;
            Push(pfrom, msgMaker.Make(NetMsgType::GETHEADERS, cs->ActiveChain().GetLocator(cs->BestHeader()), uint256()));
            LogPrint(BCLog::NET, "received header %s: missing prev block %s, sending getheaders (%d) to end (peer=%d, "
                                 "nUnconnectingHeaders=%d)\n",
                     headers[0].GetHash().ToString().c_str(), headers[0].hashPrevBlock.ToString().c_str(),
                     cs->BestHeader()->nHeight, (int)pfrom->GetId(), st->nUnconnectingHeaders);
            UpdateBlockAvailability(pfrom->GetId(), headers.back().GetHash());
            if (st->nUnconnectingHeaders % MAX_UNCONNECTING_HEADERS == 0)
                MisbehavingLocked(pfrom->GetId(), 20, "too-many-unconnected-headers");
            return true;
        }
        uint256 hashLastBlock;
        for (const CBlockHeader& h : headers) {
            if (!hashLastBlock.IsNull() && h.hashPrevBlock != hashLastBlock) {
                MisbehavingLocked(pfrom->GetId(), 20, "non-continuous headers sequence");
                return false;
            }
            hashLastBlock = h.GetHash();
        }
        received_new_header = cs->LookupBlockIndex(hashLastBlock) == nullptr;
    }
    CValidationState state;
    if (!cs->ProcessNewBlockHeaders(headers, state, &pindexLast)) {
        int nDoS;
        if (state.IsInvalid(nDoS)) {
            std::lock_guard<CCriticalSection> l(csMain());
            if (nDoS > 0) MisbehavingLocked(pfrom->GetId(), nDoS, state.GetRejectReason());
            else if (punishDuplicateInvalid) MisbehavingLocked(pfrom->GetId(), 0, state.GetRejectReason());
            return false;
        }
    }
    std::lock_guard<CCriticalSection> l(csMain());
    CNodeState* st = State(pfrom->GetId());
    if (!st) return true;
    if (st->nUnconnectingHeaders > 0)
        LogPrint(BCLog::NET, "peer=%d: resetting nUnconnectingHeaders (%d -> 0)\n", (int)pfrom->GetId(),
                 st->nUnconnectingHeaders);
    st->nUnconnectingHeaders = 0;
    if (!pindexLast) return true;
    UpdateBlockAvailability(pfrom->GetId(), pindexLast->GetBlockHash());
    if (received_new_header && pindexLast->nChainWork > cs->Tip()->nChainWork) nTimeBestReceived = GetTime();
    if (nCount == MAX_HEADERS_RESULTS) {
        // more to come
        LogPrint(BCLog::NET, "more getheaders (%d) to end to peer=%d (startheight:%d)\n", pindexLast->nHeight,
                 (int)pfrom->GetId(), (int)pfrom->nStartingHeight);
        Push(pfrom, msgMaker.Make(NetMsgType::GETHEADERS, cs->ActiveChain().GetLocator(pindexLast), uint256()));
    }
    const bool fCanDirectFetch = CanDirectFetch();
    // direct fetch of announced blocks when near the tip
    if (fCanDirectFetch && pindexLast->IsValid(BLOCK_VALID_TREE) && cs->Tip()->nChainWork <= pindexLast->nChainWork) {
        std::vector<const CBlockIndex*> vToFetch;
        const CBlockIndex* walk = pindexLast;
        while (walk && !cs->ActiveChain().Contains(walk) && vToFetch.size() <= MAX_BLOCKS_IN_TRANSIT_PER_PEER) {
            if (!(walk->nStatus & BLOCK_HAVE_DATA) && !mapBlocksInFlight.count(walk->GetBlockHash()))
                vToFetch.push_back(walk);
            walk = walk->pprev;
        }
        if (walk && !cs->ActiveChain().Contains(walk)) {
            LogPrint(BCLog::NET, "Large reorg, won't direct fetch to %s (%d)\n", pindexLast->GetBlockHash().ToString().c_str(),
                     pindexLast->nHeight);
        } else {
            std::vector<CInv> vGetData;
            for (auto r = vToFetch.rbegin(); r != vToFetch.rend(); ++r) {
                const CBlockIndex* pi = *r;
                if (st->nBlocksInFlight >= MAX_BLOCKS_IN_TRANSIT_PER_PEER) break;
                vGetData.push_back(CInv(MSG_BLOCK, pi->GetBlockHash()));
                MarkBlockAsInFlight(pfrom->GetId(), pi->GetBlockHash(), pi);
                LogPrint(BCLog::NET, "Requesting block %s from  peer=%d\n", pi->GetBlockHash().ToString().c_str(),
                         (int)pfrom->GetId());
            }
            if (vGetData.size() > 1)
                LogPrint(BCLog::NET, "Downloading blocks toward %s (%d) via headers direct fetch\n",
                         pindexLast->GetBlockHash().ToString().c_str(), pindexLast->nHeight);
            if (!vGetData.empty()) {
                if (st->fSupportsDesiredCmpctVersion && vGetData.size() == 1 && mapBlocksInFlight.size() == 1 &&
                    pindexLast->pprev->IsValid(BLOCK_VALID_CHAIN)) {
                    vGetData[0] = CInv(MSG_CMPCT_BLOCK, vGetData[0].hash);
                }
                Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, vGetData));
            }
        }
    }
    return true;
}

void PeerLogicValidation::Impl::ProcessOrphans(std::set<uint256>& work) {
    // caller holds cs_main
    std::vector<uint256> queue(work.begin(), work.end());
    std::set<NodeId> setMisbehaving;
    while (!queue.empty()) {
        const uint256 h = queue.back();
        queue.pop_back();
        std::vector<std::pair<CTransactionRef, NodeId>> candidates;
        {
            std::lock_guard<std::mutex> l(cs_orphans);
            for (uint32_t n = 0;; n++) {
                auto it = mapOrphanTransactionsByPrev.find(COutPoint(h, n));
                if (it == mapOrphanTransactionsByPrev.end()) {
                    if (n > 1000) break;
                    // outputs are sparse: scan until a gap past the highest known
                    bool any = false;
                    for (auto jt = mapOrphanTransactionsByPrev.lower_bound(COutPoint(h, n));
                         jt != mapOrphanTransactionsByPrev.end() && jt->first.hash == h; ++jt) {
                        any = true;
                        break;
                    }
                    if (!any) break;
                    continue;
                }
                for (const uint256& oh : it->second) {
                    auto ot = mapOrphanTransactions.find(oh);
                    if (ot != mapOrphanTransactions.end()) candidates.push_back({ot->second.tx, ot->second.fromPeer});
                }
            }
        }
        for (const auto& c : candidates) {
            const CTransactionRef& otx = c.first;
            const NodeId from = c.second;
            if (setMisbehaving.count(from)) continue;
            bool fMissing = false;
            CValidationState st;
            if (cs->AcceptToMemoryPool(st, otx, true, &fMissing)) {
                LogPrint(BCLog::MEMPOOL, "   accepted orphan tx %s\n", otx->GetHash().ToString().c_str());
                RelayTransaction(*otx);
                queue.push_back(otx->GetHash());
                std::lock_guard<std::mutex> l(cs_orphans);
                EraseOrphanTxLocked(otx->GetHash());
            } else if (!fMissing) {
                int nDos = 0;
                if (st.IsInvalid(nDos) && nDos > 0) {
                    MisbehavingLocked(from, nDos, "invalid orphan");
                    setMisbehaving.insert(from);
                }
                LogPrint(BCLog::MEMPOOL, "   removed orphan tx %s\n", otx->GetHash().ToString().c_str());
                recentRejects.insert(otx->GetHash());
                std::lock_guard<std::mutex> l(cs_orphans);
                EraseOrphanTxLocked(otx->GetHash());
            }
        }
    }
}

// ------------------------------------------------------------------ ProcessMessage
bool PeerLogicValidation::Impl::ProcessMessage(CNode* pfrom, const std::string& strCommand, DataStream& vRecv,
                                               int64_t nTimeReceived, std::atomic<bool>& interrupt) {
    LogPrint(BCLog::NET, "received: %s (%zu bytes) peer=%d\n", SanitizeString(strCommand).c_str(), vRecv.size(),
             (int)pfrom->GetId());
    if (gArgs.IsArgSet("-dropmessagestest") && GetRand(gArgs.GetArg("-dropmessagestest", (int64_t)0)) == 0) {
        LogPrintf("dropmessagestest DROPPING RECV MESSAGE\n");
        return true;
    }
    if (!(pfrom->GetLocalServices() & NODE_BLOOM) &&
        (strCommand == NetMsgType::FILTERLOAD || strCommand == NetMsgType::FILTERADD)) {
        if (pfrom->nVersion >= NO_BLOOM_VERSION) {
            Misbehaving(pfrom->GetId(), 100);
            return false;
        }
        pfrom->fDisconnect = true;
        return false;
    }

    if (strCommand == NetMsgType::VERSION) {
        if (pfrom->nVersion != 0) {
            Push(pfrom, CNetMsgMaker(INIT_PROTO_VERSION)
                            .Make(NetMsgType::REJECT, strCommand, (unsigned char)REJECT_DUPLICATE,
                                  std::string("Duplicate version message")));
            Misbehaving(pfrom->GetId(), 1);
            return false;
        }
        int nVersion;
        uint64_t nServiceInt;
        int64_t nTime;
        CAddress addrMe, addrFrom;
        uint64_t nNonce = 1;
        std::string strSubVer, cleanSubVer;
        int nStartingHeight = -1;
        bool fRelay = true;
        vRecv >> nVersion >> nServiceInt >> nTime >> addrMe;
        pfrom->nServices = nServiceInt;
        if (!pfrom->fInbound) connman->SetServices(pfrom->addr, nServiceInt);
        if (nVersion < MIN_PEER_PROTO_VERSION) {
            LogPrintf("peer=%d using obsolete version %i; disconnecting\n", (int)pfrom->GetId(), nVersion);
            Push(pfrom, CNetMsgMaker(INIT_PROTO_VERSION)
                            .Make(NetMsgType::REJECT, strCommand, (unsigned char)REJECT_OBSOLETE,
                                  strprintf("Version must be %d or greater", MIN_PEER_PROTO_VERSION)));
            pfrom->fDisconnect = true;
            return false;
        }
        if (nVersion == 10300) nVersion = 300;
        if (!vRecv.empty()) vRecv >> addrFrom >> nNonce;
        if (!vRecv.empty()) {
            ReadLimitedString(vRecv, strSubVer, MAX_SUBVERSION_LENGTH);
            cleanSubVer = SanitizeString(strSubVer);
        }
        if (!vRecv.empty()) vRecv >> nStartingHeight;
        if (!vRecv.empty()) vRecv >> fRelay;
        if (pfrom->fInbound && !connman->CheckIncomingNonce(nNonce)) {
            LogPrintf("connected to self at %s, disconnecting\n", pfrom->addr.ToString().c_str());
            pfrom->fDisconnect = true;
            return true;
        }
        if (pfrom->fInbound && addrMe.IsRoutable()) pfrom->SetAddrLocal(addrMe);
        if (pfrom->fInbound) PushNodeVersion(pfrom, GetAdjustedTime());
        Push(pfrom, CNetMsgMaker(INIT_PROTO_VERSION).Make(NetMsgType::VERACK));
        pfrom->nServices = nServiceInt;
        {
            std::lock_guard<std::mutex> l(pfrom->cs_SubVer);
            pfrom->strSubVer = strSubVer;
            pfrom->cleanSubVer = cleanSubVer;
        }
        pfrom->nStartingHeight = nStartingHeight;
        pfrom->fClient = !(nServiceInt & NODE_NETWORK);
        {
            std::lock_guard<std::mutex> l(pfrom->cs_filter);
            pfrom->fRelayTxes = fRelay;
        }
        pfrom->SetSendVersion(std::min(nVersion, PROTOCOL_VERSION));
        pfrom->nVersion = nVersion;
        {
            std::lock_guard<CCriticalSection> l(csMain());
            CNodeState* st = State(pfrom->GetId());
            if (st) UpdatePreferredDownload(pfrom, st);
        }
        if (!pfrom->fInbound) {
            // advertise our address and ask for theirs
            if (fListen && !cs->IsInitialBlockDownload()) {
                CAddress addr = GetLocalAddress(&pfrom->addr, pfrom->GetLocalServices());
                if (addr.IsRoutable()) {
                    pfrom->PushAddress(addr, rng);
                } else if (pfrom->GetAddrLocal().IsRoutable()) {
                    addr = CAddress(pfrom->GetAddrLocal(), pfrom->GetLocalServices());
                    addr.nTime = (uint32_t)GetAdjustedTime();
                    pfrom->PushAddress(addr, rng);
                }
            }
            if (pfrom->nVersion >= CADDR_TIME_VERSION || connman->GetAddressCount() < 1000) {
                Push(pfrom, CNetMsgMaker(pfrom->GetSendVersion()).Make(NetMsgType::GETADDR));
                pfrom->fGetAddr = true;
            }
            connman->MarkAddressGood(pfrom->addr);
        }
        LogPrintf("receive version message: %s: version %d, blocks=%d, us=%s, peer=%d%s\n", cleanSubVer.c_str(),
                  pfrom->nVersion.load(), pfrom->nStartingHeight.load(), addrMe.ToString().c_str(), (int)pfrom->GetId(),
                  fLogIPs ? (", peeraddr=" + pfrom->addr.ToString()).c_str() : "");
        const int64_t nTimeOffset = nTime - GetTime();
        pfrom->nTimeOffset = nTimeOffset;
        if (AddTimeData(pfrom->addr.ToStringIP(), nTimeOffset)) {
            SetMiscWarning(CLOCK_WARNING);
            uiInterface.ThreadSafeMessageBox(CLOCK_WARNING, "", CClientUIInterface::MSG_WARNING);
        }
        if (pfrom->fFeeler) pfrom->fDisconnect = true;
        return true;
    }

    if (pfrom->nVersion == 0) {
        // must have a version message before anything else
        Misbehaving(pfrom->GetId(), 1);
        return false;
    }

    const CNetMsgMaker msgMaker(pfrom->GetSendVersion());
    const int recvLegacyFlag = pfrom->IsLegacyBlockHeader(pfrom->GetRecvVersion()) ? SERIALIZE_BLOCK_LEGACY : 0;
    const int sendLegacyFlag = pfrom->IsLegacyBlockHeader(pfrom->GetSendVersion()) ? SERIALIZE_BLOCK_LEGACY : 0;

    if (strCommand == NetMsgType::VERACK) {
        pfrom->SetRecvVersion(std::min(pfrom->nVersion.load(), PROTOCOL_VERSION));
        if (!pfrom->fInbound) {
            std::lock_guard<CCriticalSection> l(csMain());
            if (CNodeState* st = State(pfrom->GetId())) st->fCurrentlyConnected = true;
        }
        if (pfrom->nVersion >= SENDHEADERS_VERSION) Push(pfrom, msgMaker.Make(NetMsgType::SENDHEADERS));
        if (pfrom->nVersion >= SHORT_IDS_BLOCKS_VERSION) {
            // announce support, but start in low-bandwidth mode
            bool fAnnounceUsingCMPCTBLOCK = false;
            uint64_t nCMPCTBLOCKVersion = 1;
            Push(pfrom, msgMaker.Make(NetMsgType::SENDCMPCT, fAnnounceUsingCMPCTBLOCK, nCMPCTBLOCKVersion));
        }
        pfrom->fSuccessfullyConnected = true;
        return true;
    }

    if (!pfrom->fSuccessfullyConnected) {
        Misbehaving(pfrom->GetId(), 1);
        return false;
    }

    if (strCommand == NetMsgType::ADDR) {
        std::vector<CAddress> vAddr;
        vRecv >> vAddr;
        if (pfrom->nVersion < CADDR_TIME_VERSION && connman->GetAddressCount() > 1000) return true;
        if (vAddr.size() > 1000) {
            Misbehaving(pfrom->GetId(), 20, strprintf("message addr size() = %zu", vAddr.size()));
            return false;
        }
        std::vector<CAddress> vAddrOk;
        const int64_t nNow = GetAdjustedTime();
        const int64_t nSince = nNow - 10 * 60;
        for (CAddress& addr : vAddr) {
            if (interrupt) return true;
            if ((addr.nServices & NODE_NETWORK) == 0) continue;
            if (addr.nTime <= 100000000 || addr.nTime > nNow + 10 * 60) addr.nTime = (uint32_t)(nNow - 5 * 24 * 60 * 60);
            pfrom->AddAddressKnown(addr);
            const bool fReachable = addr.IsRoutable();
            if (addr.nTime > nSince && !pfrom->fGetAddr && vAddr.size() <= 10 && addr.IsRoutable())
                RelayAddress(addr, fReachable);
            if (fReachable) vAddrOk.push_back(addr);
        }
        connman->AddNewAddresses(vAddrOk, pfrom->addr, 2 * 60 * 60);
        if (vAddr.size() < 1000) pfrom->fGetAddr = false;
        if (pfrom->fOneShot) pfrom->fDisconnect = true;
        return true;
    }

    if (strCommand == NetMsgType::SENDHEADERS) {
        std::lock_guard<CCriticalSection> l(csMain());
        if (CNodeState* st = State(pfrom->GetId())) st->fPreferHeaders = true;
        return true;
    }

    if (strCommand == NetMsgType::SENDCMPCT) {
        bool fAnnounceUsingCMPCTBLOCK = false;
        uint64_t nCMPCTBLOCKVersion = 0;
        vRecv >> fAnnounceUsingCMPCTBLOCK >> nCMPCTBLOCKVersion;
        if (nCMPCTBLOCKVersion == 1) {
            std::lock_guard<CCriticalSection> l(csMain());
            if (CNodeState* st = State(pfrom->GetId())) {
                if (!st->fProvidesHeaderAndIDs) {
                    st->fProvidesHeaderAndIDs = true;
                    st->fSupportsDesiredCmpctVersion = true;
                }
                st->fPreferHeaderAndIDs = fAnnounceUsingCMPCTBLOCK;
            }
        }
        return true;
    }

    if (strCommand == NetMsgType::INV) {
        std::vector<CInv> vInv;
        vRecv >> vInv;
        if (vInv.size() > MAX_INV_SZ) {
            Misbehaving(pfrom->GetId(), 20, strprintf("message inv size() = %zu", vInv.size()));
            return false;
        }
        bool fBlocksOnly = gArgs.GetBoolArg("-blocksonly", false);
        if (pfrom->fWhitelisted && gArgs.GetBoolArg("-whitelistrelay", true)) fBlocksOnly = false;
        std::lock_guard<CCriticalSection> l(csMain());
        std::vector<CInv> vToFetch;
        for (const CInv& inv : vInv) {
            if (interrupt) return true;
            const bool fAlreadyHave = AlreadyHave(inv);
            LogPrint(BCLog::NET, "got inv: %s  %s peer=%d\n", inv.ToString().c_str(), fAlreadyHave ? "have" : "new",
                     (int)pfrom->GetId());
            if (inv.type == MSG_BLOCK) {
                UpdateBlockAvailability(pfrom->GetId(), inv.hash);
                if (!fAlreadyHave && !mapBlocksInFlight.count(inv.hash)) {
                    // headers-first: fetch the headers leading to it
                    Push(pfrom, msgMaker.Make(NetMsgType::GETHEADERS, cs->ActiveChain().GetLocator(cs->BestHeader()),
                                              inv.hash));
                    LogPrint(BCLog::NET, "getheaders (%d) %s to peer=%d\n", cs->BestHeader()->nHeight,
                             inv.hash.ToString().c_str(), (int)pfrom->GetId());
                }
            } else {
                pfrom->AddInventoryKnown(inv);
                if (fBlocksOnly) {
                    LogPrint(BCLog::NET, "transaction (%s) inv sent in violation of protocol peer=%d\n",
                             inv.hash.ToString().c_str(), (int)pfrom->GetId());
                } else if (!fAlreadyHave && !cs->IsInitialBlockDownload()) {
                    vToFetch.push_back(inv);
                }
            }
        }
        if (!vToFetch.empty()) Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, vToFetch));
        return true;
    }

    if (strCommand == NetMsgType::GETDATA) {
        std::vector<CInv> vInv;
        vRecv >> vInv;
        if (vInv.size() > MAX_INV_SZ) {
            Misbehaving(pfrom->GetId(), 20, strprintf("message getdata size() = %zu", vInv.size()));
            return false;
        }
        LogPrint(BCLog::NET, "received getdata (%zu invsz) peer=%d\n", vInv.size(), (int)pfrom->GetId());
        std::deque<CInv>& q = mapGetData[pfrom->GetId()];
        q.insert(q.end(), vInv.begin(), vInv.end());
        ProcessGetData(pfrom, q, interrupt);
        return true;
    }

    if (strCommand == NetMsgType::GETBLOCKS) {
        CBlockLocator locator;
        uint256 hashStop;
        vRecv >> locator >> hashStop;
        {
            // a block announced by compact block may still be between its AcceptBlock and its
            // ActivateBestChain: be on the best chain before answering (reference
            // net_processing.cpp:1874-1894)
            std::shared_ptr<const CBlock> recent;
            {
                std::lock_guard<std::mutex> lr(cs_most_recent);
                recent = most_recent_block;
            }
            CValidationState dummy;
            cs->ActivateBestChain(dummy, recent);
        }
        std::lock_guard<CCriticalSection> l(csMain());
        const CBlockIndex* pi = cs->FindForkInGlobalIndex(locator);
        if (pi) pi = cs->ActiveChain().Next(pi);
        int nLimit = MAX_GETBLOCKS_RESULTS;
        std::vector<CInv> vInv;
        for (; pi; pi = cs->ActiveChain().Next(pi)) {
            if (pi->GetBlockHash() == hashStop) break;
            if (cs->PruneMode() && !(pi->nStatus & BLOCK_HAVE_DATA)) break;
            vInv.push_back(CInv(MSG_BLOCK, pi->GetBlockHash()));
            if (--nLimit <= 0) {
                pfrom->hashContinue = pi->GetBlockHash();
                break;
            }
        }
        if (!vInv.empty()) Push(pfrom, msgMaker.Make(NetMsgType::INV, vInv));
        return true;
    }

    if (strCommand == NetMsgType::GETBLOCKTXN) {
        BlockTransactionsRequest req;
        vRecv >> req;
        std::shared_ptr<const CBlock> recent;
        {
            std::lock_guard<std::mutex> lr(cs_most_recent);
            if (most_recent_block_hash == req.blockhash) recent = most_recent_block;
        }
        std::lock_guard<CCriticalSection> l(csMain());
        const CBlockIndex* pi = cs->LookupBlockIndex(req.blockhash);
        if (!pi || !(pi->nStatus & BLOCK_HAVE_DATA)) {
            LogPrintf("Peer %d sent us a getblocktxn for a block we don't have\n", (int)pfrom->GetId());
            return true;
        }
        if (pi->nHeight < cs->Height() - MAX_BLOCKTXN_DEPTH) {
            // too deep: serve the full block
            LogPrint(BCLog::NET, "Peer %d sent us a getblocktxn for a block > %i deep\n", (int)pfrom->GetId(),
                     MAX_BLOCKTXN_DEPTH);
            std::deque<CInv>& q = mapGetData[pfrom->GetId()];
            q.push_back(CInv(MSG_BLOCK, req.blockhash));
            ProcessGetData(pfrom, q, interrupt);
            return true;
        }
        CBlock block;
        if (recent) block = *recent;
        else if (!cs->ReadBlock(block, pi, false)) return true;
        BlockTransactions resp(req);
        for (size_t i = 0; i < req.indexes.size(); i++) {
            if (req.indexes[i] >= block.vtx.size()) {
                MisbehavingLocked(pfrom->GetId(), 100, "out-of-bound tx index");
                LogPrintf("Peer %d sent us a getblocktxn with out-of-bounds tx indices\n", (int)pfrom->GetId());
                return true;
            }
            resp.txn[i] = block.vtx[req.indexes[i]];
        }
        Push(pfrom, msgMaker.Make(NetMsgType::BLOCKTXN, resp));
        return true;
    }

    if (strCommand == NetMsgType::GETHEADERS) {
        CBlockLocator locator;
        uint256 hashStop;
        vRecv >> locator >> hashStop;
        std::lock_guard<CCriticalSection> l(csMain());
        if (cs->IsInitialBlockDownload() && !pfrom->fWhitelisted) {
            LogPrint(BCLog::NET, "Ignoring getheaders from peer=%d because node is in initial block download\n",
                     (int)pfrom->GetId());
            return true;
        }
        CNodeState* st = State(pfrom->GetId());
        const CBlockIndex* pi = nullptr;
        if (locator.IsNull()) {
            pi = cs->LookupBlockIndex(hashStop);
            if (!pi) return true;
        } else {
            pi = cs->FindForkInGlobalIndex(locator);
            if (pi) pi = cs->ActiveChain().Next(pi);
        }
        std::vector<CBlockHeader> vHeaders;
        int nLimit = MAX_HEADERS_RESULTS;
        for (; pi; pi = cs->ActiveChain().Next(pi)) {
            vHeaders.push_back(pi->GetBlockHeader());
            if (--nLimit <= 0 || pi->GetBlockHash() == hashStop) break;
        }
        if (st) st->pindexBestHeaderSent = pi ? pi : cs->Tip();
        Push(pfrom, msgMaker.Make(sendLegacyFlag, NetMsgType::HEADERS, HeadersForWire(vHeaders)));
        return true;
    }

    if (strCommand == NetMsgType::TX) {
        if (gArgs.GetBoolArg("-blocksonly", false) && (!pfrom->fWhitelisted || !gArgs.GetBoolArg("-whitelistrelay", true))) {
            LogPrint(BCLog::NET, "transaction sent in violation of protocol peer=%d\n", (int)pfrom->GetId());
            return true;
        }
        CMutableTransaction mtx;
        vRecv >> mtx;
        const CTransactionRef ptx = MakeTransactionRef(std::move(mtx));
        const CTransaction& tx = *ptx;
        const CInv inv(MSG_TX, tx.GetHash());
        pfrom->AddInventoryKnown(inv);
        std::lock_guard<CCriticalSection> l(csMain());
        bool fMissingInputs = false;
        CValidationState state;
        {
            std::lock_guard<std::mutex> li(pfrom->cs_inventory);
            for (auto it = pfrom->mapAskFor.begin(); it != pfrom->mapAskFor.end();)
                if (it->second.hash == inv.hash) it = pfrom->mapAskFor.erase(it);
                else ++it;
            pfrom->setAskFor.erase(inv.hash);
        }
        {
            std::lock_guard<std::mutex> la(cs_mapAlreadyAskedFor);
            mapAlreadyAskedFor.erase(inv.hash);
        }
        if (!AlreadyHave(inv) && cs->AcceptToMemoryPool(state, ptx, true, &fMissingInputs)) {
            RelayTransaction(tx);
            LogPrint(BCLog::MEMPOOL, "AcceptToMemoryPool: peer=%d: accepted %s (poolsz %lu txn, %lu kB)\n",
                     (int)pfrom->GetId(), tx.GetHash().ToString().c_str(), pool->size(),
                     (unsigned long)(pool->DynamicMemoryUsage() / 1000));
            std::set<uint256> work{tx.GetHash()};
            ProcessOrphans(work);
        } else if (fMissingInputs) {
            bool fRejectedParents = false;
            for (const CTxIn& in : tx.vin)
                if (recentRejects.contains(in.prevout.hash)) {
                    fRejectedParents = true;
                    break;
                }
            if (!fRejectedParents) {
                for (const CTxIn& in : tx.vin) {
                    const CInv pinv(MSG_TX, in.prevout.hash);
                    pfrom->AddInventoryKnown(pinv);
                    if (!AlreadyHave(pinv)) pfrom->AskFor(pinv);
                }
                AddOrphanTx(ptx, pfrom->GetId());
                const unsigned nMaxOrphanTx =
                    (unsigned)std::max<int64_t>(0, gArgs.GetArg("-maxorphantx", (int64_t)DEFAULT_MAX_ORPHAN_TRANSACTIONS));
                const unsigned nEvicted = LimitOrphanTxSize(nMaxOrphanTx);
                if (nEvicted > 0) LogPrint(BCLog::MEMPOOL, "mapOrphan overflow, removed %u tx\n", nEvicted);
            } else {
                LogPrint(BCLog::MEMPOOL, "not keeping orphan with rejected parents %s\n", tx.GetHash().ToString().c_str());
                recentRejects.insert(tx.GetHash());
            }
        } else {
            if (!state.CorruptionPossible()) {
                recentRejects.insert(tx.GetHash());
                if (state.GetRejectCode() != REJECT_INSUFFICIENTFEE) AddToCompactExtraTransactions(ptx);
            }
            if (pfrom->fWhitelisted && gArgs.GetBoolArg("-whitelistforcerelay", true)) {
                int nDoS = 0;
                if (!state.IsInvalid(nDoS) || nDoS == 0) {
                    LogPrintf("Force relaying tx %s from whitelisted peer=%d\n", tx.GetHash().ToString().c_str(),
                              (int)pfrom->GetId());
                    RelayTransaction(tx);
                }
            }
        }
        int nDoS = 0;
        if (state.IsInvalid(nDoS)) {
            LogPrint(BCLog::MEMPOOLREJ, "%s from peer=%d was not accepted: %s\n", tx.GetHash().ToString().c_str(),
                     (int)pfrom->GetId(), FormatStateMessage(state).c_str());
            if (state.GetRejectCode() > 0 && state.GetRejectCode() < REJECT_INTERNAL)
                Push(pfrom, msgMaker.Make(NetMsgType::REJECT, strCommand, (unsigned char)state.GetRejectCode(),
                                          state.GetRejectReason().substr(0, MAX_REJECT_MESSAGE_LENGTH), inv.hash));
            if (nDoS > 0) MisbehavingLocked(pfrom->GetId(), nDoS, state.GetRejectReason());
        }
        return true;
    }

    if (strCommand == NetMsgType::CMPCTBLOCK) {
        vRecv.SetVersion(vRecv.GetVersion() | recvLegacyFlag);
        CBlockHeaderAndShortTxIDs cmpctblock;
        vRecv >> cmpctblock;
        bool received_new_header = false;
        {
            std::lock_guard<CCriticalSection> l(csMain());
            if (!cs->LookupBlockIndex(cmpctblock.header.hashPrevBlock)) {
                // doesn't connect: ask for headers
                if (!cs->IsInitialBlockDownload())
                    Push(pfrom, msgMaker.Make(NetMsgType::GETHEADERS, cs->ActiveChain().GetLocator(cs->BestHeader()),
                                              uint256()));
                return true;
            }
            if (!cs->LookupBlockIndex(cmpctblock.header.GetHash())) received_new_header = true;
        }
        const CBlockIndex* pindex = nullptr;
        CValidationState state;
        if (!cs->ProcessNewBlockHeaders({cmpctblock.header}, state, &pindex)) {
            int nDoS;
            if (state.IsInvalid(nDoS)) {
                if (nDoS > 0) Misbehaving(pfrom->GetId(), nDoS, state.GetRejectReason());
                else LogPrint(BCLog::NET, "Peer %d sent us invalid header via cmpctblock\n", (int)pfrom->GetId());
                return true;
            }
        }
        bool fProcessBLOCKTXN = false;
        DataStream blockTxnMsg;
        bool fRevertToHeaderProcessing = false;
        bool fBlockReconstructed = false;
        std::shared_ptr<CBlock> pblock = std::make_shared<CBlock>();
        {
            std::lock_guard<CCriticalSection> l(csMain());
            if (!pindex) return true;
            UpdateBlockAvailability(pfrom->GetId(), pindex->GetBlockHash());
            CNodeState* st = State(pfrom->GetId());
            if (received_new_header && pindex->nChainWork > cs->Tip()->nChainWork) nTimeBestReceived = GetTime();
            auto blockInFlightIt = mapBlocksInFlight.find(pindex->GetBlockHash());
            const bool fAlreadyInFlight = blockInFlightIt != mapBlocksInFlight.end();
            if (pindex->nStatus & BLOCK_HAVE_DATA) return true;
            if (pindex->nChainWork <= cs->Tip()->nChainWork || pindex->nTx != 0) {
                if (fAlreadyInFlight) {
                    std::vector<CInv> vInv{CInv(MSG_BLOCK, cmpctblock.header.GetHash())};
                    Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, vInv));
                }
                return true;
            }
            if (!fAlreadyInFlight && !CanDirectFetch()) return true;
            if (pindex->nHeight <= cs->Height() + 2) {
                if ((!fAlreadyInFlight && st->nBlocksInFlight < MAX_BLOCKS_IN_TRANSIT_PER_PEER) ||
                    (fAlreadyInFlight && blockInFlightIt->second.first == pfrom->GetId())) {
                    std::list<QueuedBlock>::iterator* queuedBlockIt = nullptr;
                    if (!MarkBlockAsInFlight(pfrom->GetId(), pindex->GetBlockHash(), pindex, &queuedBlockIt)) {
                        if (!(*queuedBlockIt)->partialBlock)
                            (*queuedBlockIt)->partialBlock.reset(new PartiallyDownloadedBlock(pool));
                        else {
                            LogPrint(BCLog::NET, "Peer sent us compact block we were already syncing!\n");
                            return true;
                        }
                    }
                    PartiallyDownloadedBlock& partial = *(*queuedBlockIt)->partialBlock;
                    std::vector<std::pair<uint256, CTransactionRef>> extra;
                    for (const auto& e : vExtraTxnForCompact)
                        if (e.second) extra.push_back(e);
                    const ReadStatus status = partial.InitData(cmpctblock, extra);
                    if (status == READ_STATUS_INVALID) {
                        MarkBlockAsReceived(pindex->GetBlockHash());
                        MisbehavingLocked(pfrom->GetId(), 100, "invalid compact block");
                        return true;
                    } else if (status == READ_STATUS_FAILED) {
                        std::vector<CInv> vInv{CInv(MSG_BLOCK, cmpctblock.header.GetHash())};
                        Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, vInv));
                        return true;
                    }
                    BlockTransactionsRequest req;
                    for (size_t i = 0; i < cmpctblock.BlockTxCount(); i++)
                        if (!partial.IsTxAvailable(i)) req.indexes.push_back((uint16_t)i);
                    if (req.indexes.empty()) {
                        // everything was in the mempool: treat as an empty blocktxn
                        BlockTransactions txn;
                        txn.blockhash = cmpctblock.header.GetHash();
                        blockTxnMsg << txn;
                        fProcessBLOCKTXN = true;
                    } else {
                        req.blockhash = pindex->GetBlockHash();
                        Push(pfrom, msgMaker.Make(NetMsgType::GETBLOCKTXN, req));
                    }
                } else {
                    // already in flight from another peer: try a mempool-only reconstruction
                    PartiallyDownloadedBlock tempBlock(pool);
                    const ReadStatus status = tempBlock.InitData(cmpctblock, {});
                    if (status != READ_STATUS_OK) return true;
                    std::vector<CTransactionRef> dummy;
                    if (tempBlock.FillBlock(*pblock, dummy) == READ_STATUS_OK) fBlockReconstructed = true;
                }
            } else {
                if (fAlreadyInFlight) {
                    std::vector<CInv> vInv{CInv(MSG_BLOCK, cmpctblock.header.GetHash())};
                    Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, vInv));
                    return true;
                }
                fRevertToHeaderProcessing = true;
            }
        }
        if (fProcessBLOCKTXN) return ProcessMessage(pfrom, NetMsgType::BLOCKTXN, blockTxnMsg, nTimeReceived, interrupt);
        if (fRevertToHeaderProcessing) return ProcessHeadersMessage(pfrom, {cmpctblock.header}, true);
        if (fBlockReconstructed) {
            {
                std::lock_guard<CCriticalSection> l(csMain());
                mapBlockSource.emplace(pblock->GetHash(), std::make_pair(pfrom->GetId(), false));
            }
            bool fNewBlock = false;
            cs->ProcessNewBlock(pblock, true, &fNewBlock);
            if (fNewBlock) pfrom->nLastBlockTime = GetTime();
            std::lock_guard<CCriticalSection> l(csMain());
            if (pindex->IsValid(BLOCK_VALID_TRANSACTIONS)) MarkBlockAsReceived(pblock->GetHash());
        }
        return true;
    }

    if (strCommand == NetMsgType::BLOCKTXN) {
        BlockTransactions resp;
        vRecv >> resp;
        std::shared_ptr<CBlock> pblock = std::make_shared<CBlock>();
        bool fBlockRead = false;
        {
            std::lock_guard<CCriticalSection> l(csMain());
            auto it = mapBlocksInFlight.find(resp.blockhash);
            if (it == mapBlocksInFlight.end() || !it->second.second->partialBlock ||
                it->second.first != pfrom->GetId()) {
                LogPrint(BCLog::NET, "Peer %d sent us block transactions for block we weren't expecting\n",
                         (int)pfrom->GetId());
                return true;
            }
            PartiallyDownloadedBlock& partial = *it->second.second->partialBlock;
            const ReadStatus status = partial.FillBlock(*pblock, resp.txn);
            if (status == READ_STATUS_INVALID) {
                MarkBlockAsReceived(resp.blockhash);
                MisbehavingLocked(pfrom->GetId(), 100, "invalid compact block/non-matching block transactions");
                return true;
            } else if (status == READ_STATUS_FAILED) {
                // possible short-id collision (merkle mismatch): fetch the full block
                // (reference net_processing.cpp BLOCKTXN; CHECKBLOCK_FAILED is processed below)
                std::vector<CInv> invs{CInv(MSG_BLOCK, resp.blockhash)};
                Push(pfrom, msgMaker.Make(NetMsgType::GETDATA, invs));
            } else {
                MarkBlockAsReceived(resp.blockhash);
                fBlockRead = true;
                mapBlockSource.emplace(resp.blockhash, std::make_pair(pfrom->GetId(), false));
            }
        }
        if (fBlockRead) {
            bool fNewBlock = false;
            cs->ProcessNewBlock(pblock, true, &fNewBlock);
            if (fNewBlock) pfrom->nLastBlockTime = GetTime();
        }
        return true;
    }

    if (strCommand == NetMsgType::HEADERS) {
        vRecv.SetVersion(vRecv.GetVersion() | recvLegacyFlag);
        std::vector<CBlockHeader> headers;
        const uint64_t nCount = ReadCompactSize(vRecv);
        if (nCount > MAX_HEADERS_RESULTS) {
            Misbehaving(pfrom->GetId(), 20, strprintf("headers message size = %u", (unsigned)nCount));
            return false;
        }
        headers.resize(nCount);
        for (uint64_t n = 0; n < nCount; n++) {
            vRecv >> headers[n];
            ReadCompactSize(vRecv); // ignore tx count; assume 0
        }
        return ProcessHeadersMessage(pfrom, headers, false);
    }

    if (strCommand == NetMsgType::BLOCK) {
        vRecv.SetVersion(vRecv.GetVersion() | recvLegacyFlag);
        std::shared_ptr<CBlock> pblock = std::make_shared<CBlock>();
        vRecv >> *pblock;
        LogPrint(BCLog::NET, "received block %s peer=%d\n", pblock->GetHash().ToString().c_str(), (int)pfrom->GetId());
        // whitelisted peers may push blocks unrequested outside IBD (reference
        // src/net_processing.cpp BLOCK handler: fWhitelisted && !IsInitialBlockDownload())
        bool forceProcessing = pfrom->fWhitelisted && !cs->IsInitialBlockDownload();
        const uint256 hash = pblock->GetHash();
        {
            std::lock_guard<CCriticalSection> l(csMain());
            forceProcessing |= MarkBlockAsReceived(hash);
            mapBlockSource.emplace(hash, std::make_pair(pfrom->GetId(), true));
        }
        bool fNewBlock = false;
        cs->ProcessNewBlock(pblock, forceProcessing, &fNewBlock);
        if (fNewBlock) pfrom->nLastBlockTime = GetTime();
        return true;
    }

    if (strCommand == NetMsgType::GETADDR) {
        // inbound only, once per connection (fingerprinting protection)
        if (!pfrom->fInbound) {
            LogPrint(BCLog::NET, "Ignoring \"getaddr\" from outbound connection. peer=%d\n", (int)pfrom->GetId());
            return true;
        }
        if (pfrom->fSentAddr) {
            LogPrint(BCLog::NET, "Ignoring repeated \"getaddr\". peer=%d\n", (int)pfrom->GetId());
            return true;
        }
        pfrom->fSentAddr = true;
        pfrom->vAddrToSend.clear();
        for (const CAddress& a : connman->GetAddresses()) pfrom->PushAddress(a, rng);
        return true;
    }

    if (strCommand == NetMsgType::MEMPOOL) {
        if (!(pfrom->GetLocalServices() & NODE_BLOOM) && !pfrom->fWhitelisted) {
            LogPrint(BCLog::NET, "mempool request with bloom filters disabled, disconnect peer=%d\n", (int)pfrom->GetId());
            pfrom->fDisconnect = true;
            return true;
        }
        if (connman->OutboundTargetReached(false) && !pfrom->fWhitelisted) {
            LogPrint(BCLog::NET, "mempool request with bandwidth limit reached, disconnect peer=%d\n", (int)pfrom->GetId());
            pfrom->fDisconnect = true;
            return true;
        }
        std::lock_guard<std::mutex> l(pfrom->cs_inventory);
        pfrom->fSendMempool = true;
        return true;
    }

    if (strCommand == NetMsgType::PING) {
        if (pfrom->nVersion > BIP0031_VERSION) {
            uint64_t nonce = 0;
            vRecv >> nonce;
            Push(pfrom, msgMaker.Make(NetMsgType::PONG, nonce));
        }
        return true;
    }

    if (strCommand == NetMsgType::PONG) {
        const int64_t pingUsecEnd = nTimeReceived;
        uint64_t nonce = 0;
        const size_t nAvail = vRecv.size();
        bool bPingFinished = false;
        std::string sProblem;
        if (nAvail >= sizeof(nonce)) {
            vRecv >> nonce;
            if (pfrom->nPingNonceSent != 0) {
                if (nonce == pfrom->nPingNonceSent) {
                    bPingFinished = true;
                    const int64_t pingUsecTime = pingUsecEnd - pfrom->nPingUsecStart;
                    if (pingUsecTime > 0) {
                        pfrom->nPingUsecTime = pingUsecTime;
                        pfrom->nMinPingUsecTime = std::min(pfrom->nMinPingUsecTime.load(), pingUsecTime);
                    } else {
                        sProblem = "Timing mishap";
                    }
                } else {
                    sProblem = "Nonce mismatch";
                    if (nonce == 0) {
                        bPingFinished = true;
                        sProblem = "Nonce zero";
                    }
                }
            } else {
                sProblem = "Unsolicited pong without ping";
            }
        } else {
            bPingFinished = true;
            sProblem = "Short payload";
        }
        if (!sProblem.empty())
            LogPrint(BCLog::NET, "pong peer=%d: %s, %x expected, %x received, %zu bytes\n", (int)pfrom->GetId(),
                     sProblem.c_str(), (unsigned)pfrom->nPingNonceSent, (unsigned)nonce, nAvail);
        if (bPingFinished) pfrom->nPingNonceSent = 0;
        return true;
    }

    if (strCommand == NetMsgType::FILTERLOAD) {
        CBloomFilter filter;
        vRecv >> filter;
        if (!filter.IsWithinSizeConstraints()) {
            Misbehaving(pfrom->GetId(), 100, "oversized bloom filter");
        } else {
            std::lock_guard<std::mutex> l(pfrom->cs_filter);
            pfrom->pfilter.reset(new CBloomFilter(filter));
            pfrom->pfilter->UpdateEmptyFull();
            pfrom->fRelayTxes = true;
        }
        return true;
    }

    if (strCommand == NetMsgType::FILTERADD) {
        std::vector<unsigned char> vData;
        vRecv >> vData;
        bool bad = false;
        if (vData.size() > MAX_SCRIPT_ELEMENT_SIZE) {
            bad = true;
        } else {
            std::lock_guard<std::mutex> l(pfrom->cs_filter);
            if (pfrom->pfilter) pfrom->pfilter->insert(vData);
            else bad = true;
        }
        if (bad) Misbehaving(pfrom->GetId(), 100, "bad filteradd");
        return true;
    }

    if (strCommand == NetMsgType::FILTERCLEAR) {
        std::lock_guard<std::mutex> l(pfrom->cs_filter);
        if (pfrom->GetLocalServices() & NODE_BLOOM) pfrom->pfilter.reset(new CBloomFilter());
        pfrom->fRelayTxes = true;
        return true;
    }

    if (strCommand == NetMsgType::FEEFILTER) {
        int64_t newFeeFilter = 0;
        vRecv >> newFeeFilter;
        if (MoneyRange(newFeeFilter)) {
            pfrom->minFeeFilter = newFeeFilter;
            LogPrint(BCLog::NET, "received: feefilter of %s from peer=%d\n", CFeeRate(newFeeFilter).ToString().c_str(),
                     (int)pfrom->GetId());
        }
        return true;
    }

    if (strCommand == NetMsgType::REJECT) {
        if (LogAcceptCategory(BCLog::NET)) {
            try {
                std::string strMsg, strReason;
                unsigned char ccode;
                ReadLimitedString(vRecv, strMsg, CMessageHeader::COMMAND_SIZE);
                vRecv >> ccode;
                ReadLimitedString(vRecv, strReason, MAX_REJECT_MESSAGE_LENGTH);
                std::string ss = strMsg + " code " + std::to_string(ccode) + ": " + strReason;
                if (strMsg == NetMsgType::BLOCK || strMsg == NetMsgType::TX) {
                    uint256 hash;
                    vRecv >> hash;
                    ss += ": hash " + hash.ToString();
                }
                LogPrint(BCLog::NET, "Reject %s\n", SanitizeString(ss).c_str());
            } catch (const std::exception&) {
                LogPrint(BCLog::NET, "Unparseable reject message received\n");
            }
        }
        return true;
    }

    if (strCommand == NetMsgType::NOTFOUND) return true;

    LogPrint(BCLog::NET, "Unknown command \"%s\" from peer=%d\n", SanitizeString(strCommand).c_str(), (int)pfrom->GetId());
    return true;
}

bool PeerLogicValidation::Impl::SendRejectsAndCheckIfBanned(CNode* pnode) {
    CNodeState* st = State(pnode->GetId());
    if (!st) return false;
    for (const CNodeState::Reject& r : st->rejects)
        Push(pnode, CNetMsgMaker(INIT_PROTO_VERSION)
                        .Make(NetMsgType::REJECT, std::string(NetMsgType::BLOCK), r.code, r.reason, r.hash));
    st->rejects.clear();
    if (st->fShouldBan) {
        st->fShouldBan = false;
        if (pnode->fWhitelisted) {
            LogPrintf("Warning: not punishing whitelisted peer %s!\n", pnode->addr.ToString().c_str());
        } else if (pnode->fAddnode) {
            LogPrintf("Warning: not punishing addnoded peer %s!\n", pnode->addr.ToString().c_str());
        } else {
            pnode->fDisconnect = true;
            if (pnode->addr.IsLocal()) {
                LogPrintf("Warning: not banning local peer %s!\n", pnode->addr.ToString().c_str());
            } else {
                connman->Ban(pnode->addr, BanReasonNodeMisbehaving);
            }
        }
        return true;
    }
    return false;
}

bool PeerLogicValidation::ProcessMessages(CNode* pfrom, std::atomic<bool>& interrupt) {
    bool fMoreWork = false;
    {
        std::lock_guard<CCriticalSection> l(impl->csMain());
        auto it = impl->mapGetData.find(pfrom->GetId());
        if (it != impl->mapGetData.end() && !it->second.empty()) impl->ProcessGetData(pfrom, it->second, interrupt);
        if (it != impl->mapGetData.end() && !it->second.empty()) return true;
    }
    if (pfrom->fDisconnect) return false;
    if (pfrom->fPauseSend) return false;
    std::list<CNetMessage> msgs;
    {
        std::lock_guard<std::mutex> l(pfrom->cs_vProcessMsg);
        if (pfrom->vProcessMsg.empty()) return false;
        msgs.splice(msgs.begin(), pfrom->vProcessMsg, pfrom->vProcessMsg.begin());
        pfrom->nProcessQueueSize -= msgs.front().payload.size() + CMessageHeader::HEADER_SIZE;
        pfrom->fPauseRecv = pfrom->nProcessQueueSize > impl->connman->GetReceiveFloodSize();
        fMoreWork = !pfrom->vProcessMsg.empty();
    }
    CNetMessage& msg = msgs.front();
    const std::string strCommand = msg.hdr.GetCommand();
    DataStream vRecv(msg.payload, SER_NETWORK, pfrom->GetRecvVersion());
    bool fRet = false;
    try {
        fRet = impl->ProcessMessage(pfrom, strCommand, vRecv, msg.nTime, interrupt);
        if (interrupt) return false;
        {
            std::lock_guard<CCriticalSection> l(impl->csMain());
            auto it = impl->mapGetData.find(pfrom->GetId());
            if (it != impl->mapGetData.end() && !it->second.empty()) fMoreWork = true;
        }
    } catch (const std::ios_base::failure& e) {
        impl->Push(pfrom, CNetMsgMaker(INIT_PROTO_VERSION)
                              .Make(NetMsgType::REJECT, strCommand, (unsigned char)REJECT_MALFORMED,
                                    std::string("error parsing message")));
        LogPrintf("%s(%s, %u bytes): Exception '%s' caught\n", __func__, SanitizeString(strCommand).c_str(),
                  msg.hdr.nMessageSize, e.what());
    } catch (const std::exception& e) {
        LogPrintf("%s(%s, %u bytes): Exception '%s' caught\n", __func__, SanitizeString(strCommand).c_str(),
                  msg.hdr.nMessageSize, e.what());
    }
    if (!fRet)
        LogPrint(BCLog::NET, "%s(%s, %u bytes) FAILED peer=%d\n", __func__, SanitizeString(strCommand).c_str(),
                 msg.hdr.nMessageSize, (int)pfrom->GetId());
    std::lock_guard<CCriticalSection> l(impl->csMain());
    impl->SendRejectsAndCheckIfBanned(pfrom);
    return fMoreWork;
}

// ------------------------------------------------------------------ SendMessages
bool PeerLogicValidation::SendMessages(CNode* pto, std::atomic<bool>& interrupt) {
    if (!pto->fSuccessfullyConnected || pto->fDisconnect) return true;
    Impl& I = *impl;
    const CNetMsgMaker msgMaker(pto->GetSendVersion());
    const int legacyFlag = pto->IsLegacyBlockHeader(pto->GetSendVersion()) ? SERIALIZE_BLOCK_LEGACY : 0;

    // ---- ping
    bool pingSend = false;
    if (pto->fPingQueued) pingSend = true;
    if (pto->nPingNonceSent == 0 && pto->nPingUsecStart + PING_INTERVAL * 1000000LL < GetTimeMicros()) pingSend = true;
    if (pingSend) {
        uint64_t nonce = 0;
        while (nonce == 0) GetRandBytes((unsigned char*)&nonce, sizeof(nonce));
        pto->fPingQueued = false;
        pto->nPingUsecStart = GetTimeMicros();
        if (pto->nVersion > BIP0031_VERSION) {
            pto->nPingNonceSent = nonce;
            I.Push(pto, msgMaker.Make(NetMsgType::PING, nonce));
        } else {
            pto->nPingNonceSent = 0;
            I.Push(pto, msgMaker.Make(NetMsgType::PING));
        }
    }

    std::unique_lock<CCriticalSection> lockMain(I.csMain(), std::try_to_lock);
    if (!lockMain) return true; // busy validating: try again next round
    AssertLockHeld(I.csMain());   // (unique_lock is invisible to the thread-safety analysis)
    if (I.SendRejectsAndCheckIfBanned(pto)) return true;
    CNodeState* st = I.State(pto->GetId());
    if (!st) return true;

    const int64_t nNow = GetTimeMicros();
    // ---- address refresh / broadcast
    if (!I.cs->IsInitialBlockDownload() && pto->nNextLocalAddrSend < nNow) {
        CAddress addr = GetLocalAddress(&pto->addr, pto->GetLocalServices());
        if (addr.IsRoutable()) pto->PushAddress(addr, I.rng);
        pto->nNextLocalAddrSend = PoissonNextSend(nNow, 24 * 60 * 60);
    }
    if (pto->nNextAddrSend < nNow) {
        pto->nNextAddrSend = PoissonNextSend(nNow, 30);
        std::vector<CAddress> vAddr;
        vAddr.reserve(pto->vAddrToSend.size());
        for (const CAddress& a : pto->vAddrToSend) {
            if (!pto->addrKnown.contains(a.GetKey())) {
                pto->addrKnown.insert(a.GetKey());
                vAddr.push_back(a);
                if (vAddr.size() >= 1000) {
                    I.Push(pto, msgMaker.Make(NetMsgType::ADDR, vAddr));
                    vAddr.clear();
                }
            }
        }
        pto->vAddrToSend.clear();
        if (!vAddr.empty()) I.Push(pto, msgMaker.Make(NetMsgType::ADDR, vAddr));
        if (pto->vAddrToSend.capacity() > 40) pto->vAddrToSend.shrink_to_fit();
    }

    // ---- start headers sync
    I.ProcessBlockAvailability(pto->GetId());
    const CBlockIndex* bestHeader = I.cs->BestHeader();
    const bool fFetch = st->fPreferredDownload || (I.nPreferredDownload == 0 && !pto->fClient && !pto->fOneShot);
    if (!st->fSyncStarted && !pto->fClient && bestHeader) {
        if ((I.nSyncStarted == 0 && fFetch) ||
            bestHeader->GetBlockTime() > GetAdjustedTime() - 24 * 60 * 60) {
            st->fSyncStarted = true;
            I.nSyncStarted++;
            const CBlockIndex* pindexStart = bestHeader->pprev ? bestHeader->pprev : bestHeader;
            LogPrint(BCLog::NET, "initial getheaders (%d) to peer=%d (startheight:%d)\n", pindexStart->nHeight,
                     (int)pto->GetId(), (int)pto->nStartingHeight);
            I.Push(pto, msgMaker.Make(NetMsgType::GETHEADERS, I.cs->ActiveChain().GetLocator(pindexStart), uint256()));
        }
    }

    // ---- block announcements
    {
        std::vector<uint256> toAnnounce;
        {
            std::lock_guard<std::mutex> li(pto->cs_inventory);
            toAnnounce.swap(pto->vBlockHashesToAnnounce);
        }
        std::vector<CBlockHeader> vHeaders;
        bool fRevertToInv = (!st->fPreferHeaders && (!st->fPreferHeaderAndIDs || toAnnounce.size() > 1)) ||
                            toAnnounce.size() > MAX_BLOCKS_TO_ANNOUNCE;
        const CBlockIndex* pBestIndex = nullptr;
        if (!fRevertToInv) {
            bool fFoundStartingHeader = false;
            for (const uint256& h : toAnnounce) {
                const CBlockIndex* pi = I.cs->LookupBlockIndex(h);
                if (!pi) continue;
                if (!I.cs->ActiveChain().Contains(pi)) {
                    fRevertToInv = true;
                    break;
                }
                if (pBestIndex && pi->pprev != pBestIndex) {
                    fRevertToInv = true;
                    break;
                }
                pBestIndex = pi;
                if (fFoundStartingHeader) {
                    vHeaders.push_back(pi->GetBlockHeader());
                } else if (I.PeerHasHeader(st, pi)) {
                    continue;
                } else if (!pi->pprev || I.PeerHasHeader(st, pi->pprev)) {
                    fFoundStartingHeader = true;
                    vHeaders.push_back(pi->GetBlockHeader());
                } else {
                    fRevertToInv = true;
                    break;
                }
            }
        }
        if (!fRevertToInv && !vHeaders.empty()) {
            if (vHeaders.size() == 1 && st->fPreferHeaderAndIDs) {
                bool fGotBlockFromCache = false;
                {
                    std::lock_guard<std::mutex> lr(I.cs_most_recent);
                    if (I.most_recent_block_hash == pBestIndex->GetBlockHash()) {
                        I.Push(pto, msgMaker.Make(legacyFlag, NetMsgType::CMPCTBLOCK, *I.most_recent_compact_block));
                        fGotBlockFromCache = true;
                    }
                }
                if (!fGotBlockFromCache) {
                    CBlock block;
                    if (I.cs->ReadBlock(block, pBestIndex, false)) {
                        CBlockHeaderAndShortTxIDs cmpct(block, I.rng.rand64());
                        I.Push(pto, msgMaker.Make(legacyFlag, NetMsgType::CMPCTBLOCK, cmpct));
                    }
                }
                st->pindexBestHeaderSent = pBestIndex;
            } else if (st->fPreferHeaders) {
                I.Push(pto, msgMaker.Make(legacyFlag, NetMsgType::HEADERS, HeadersForWire(vHeaders)));
                st->pindexBestHeaderSent = pBestIndex;
            } else {
                fRevertToInv = true;
            }
        }
        if (fRevertToInv && !toAnnounce.empty()) {
            // announce only the tip by inv
            const uint256& h = toAnnounce.back();
            const CBlockIndex* pi = I.cs->LookupBlockIndex(h);
            if (pi && I.cs->ActiveChain().Contains(pi)) {
                if (!I.PeerHasHeader(st, pi)) pto->PushInventory(CInv(MSG_BLOCK, h));
            }
        }
    }

    // ---- inventory
    std::vector<CInv> vInv;
    {
        std::lock_guard<std::mutex> li(pto->cs_inventory);
        vInv.reserve(std::max<size_t>(pto->vInventoryBlockToSend.size(), INVENTORY_BROADCAST_MAX));
        for (const uint256& h : pto->vInventoryBlockToSend) {
            vInv.push_back(CInv(MSG_BLOCK, h));
            if (vInv.size() == MAX_INV_SZ) {
                I.Push(pto, msgMaker.Make(NetMsgType::INV, vInv));
                vInv.clear();
            }
        }
        pto->vInventoryBlockToSend.clear();

        bool fSendTrickle = pto->fWhitelisted;
        if (pto->nNextInvSend < nNow) {
            fSendTrickle = true;
            pto->nNextInvSend = pto->fInbound ? I.connman->PoissonNextSendInbound(nNow, INVENTORY_BROADCAST_INTERVAL)
                                              : PoissonNextSend(nNow, INVENTORY_BROADCAST_INTERVAL >> 1);
        }
        bool fRelay;
        {
            std::lock_guard<std::mutex> lf(pto->cs_filter);
            fRelay = pto->fRelayTxes;
        }
        if (fSendTrickle && !fRelay) pto->setInventoryTxToSend.clear();
        if (fSendTrickle && pto->fSendMempool) {
            pto->fSendMempool = false;
            const Amount filterrate = pto->minFeeFilter;
            std::lock_guard<std::mutex> lf(pto->cs_filter);
            for (const TxMempoolInfo& txinfo : I.pool->infoAll()) {
                const uint256& h = txinfo.tx->GetHash();
                pto->setInventoryTxToSend.erase(h);
                if (filterrate && txinfo.feeRate.GetFeePerK() < filterrate) continue;
                if (pto->pfilter && !pto->pfilter->IsRelevantAndUpdate(*txinfo.tx)) continue;
                pto->filterInventoryKnown.insert(h);
                vInv.push_back(CInv(MSG_TX, h));
                if (vInv.size() == MAX_INV_SZ) {
                    I.Push(pto, msgMaker.Make(NetMsgType::INV, vInv));
                    vInv.clear();
                }
            }
            pto->timeLastMempoolReq = GetTime();
        }
        if (fSendTrickle) {
            std::vector<uint256> vInvTx(pto->setInventoryTxToSend.begin(), pto->setInventoryTxToSend.end());
            const Amount filterrate = pto->minFeeFilter;
            // topological-ish order: ancestors first (by ancestor count), then fee
            std::sort(vInvTx.begin(), vInvTx.end(), [&](const uint256& a, const uint256& b) {
                const CTxMemPoolEntry* ea = I.pool->GetEntry(a);
                const CTxMemPoolEntry* eb = I.pool->GetEntry(b);
                if (!ea || !eb) return ea != nullptr;
                if (ea->GetCountWithAncestors() != eb->GetCountWithAncestors())
                    return ea->GetCountWithAncestors() < eb->GetCountWithAncestors();
                return ea->GetModifiedFee() * (int64_t)eb->GetTxSize() > eb->GetModifiedFee() * (int64_t)ea->GetTxSize();
            });
            unsigned nRelayedTransactions = 0;
            std::lock_guard<std::mutex> lf(pto->cs_filter);
            for (const uint256& h : vInvTx) {
                if (nRelayedTransactions >= INVENTORY_BROADCAST_MAX) break;
                pto->setInventoryTxToSend.erase(h);
                if (pto->filterInventoryKnown.contains(h)) continue;
                TxMempoolInfo txinfo = I.pool->info(h);
                if (!txinfo.tx) continue;
                if (filterrate && txinfo.feeRate.GetFeePerK() < filterrate) continue;
                if (pto->pfilter && !pto->pfilter->IsRelevantAndUpdate(*txinfo.tx)) continue;
                vInv.push_back(CInv(MSG_TX, h));
                nRelayedTransactions++;
                if (vInv.size() == MAX_INV_SZ) {
                    I.Push(pto, msgMaker.Make(NetMsgType::INV, vInv));
                    vInv.clear();
                }
                pto->filterInventoryKnown.insert(h);
            }
        }
    }
    if (!vInv.empty()) I.Push(pto, msgMaker.Make(NetMsgType::INV, vInv));

    // ---- stalling / download timeouts
    const Consensus::Params& consensus = I.cs->Params().GetConsensus();
    if (st->nStallingSince && st->nStallingSince < nNow - 1000000LL * BLOCK_STALLING_TIMEOUT) {
        LogPrintf("Peer=%d is stalling block download, disconnecting\n", (int)pto->GetId());
        pto->fDisconnect = true;
        return true;
    }
    if (!st->vBlocksInFlight.empty()) {
        const QueuedBlock& qb = st->vBlocksInFlight.front();
        const int nOtherPeersWithValidatedDownloads = I.nPeersWithValidatedDownloads - (st->nBlocksInFlightValidHeaders > 0);
        if (nNow > st->nDownloadingSince + consensus.nPowTargetSpacing * (BLOCK_DOWNLOAD_TIMEOUT_BASE +
                                                                           BLOCK_DOWNLOAD_TIMEOUT_PER_PEER *
                                                                               nOtherPeersWithValidatedDownloads)) {
            LogPrintf("Timeout downloading block %s from peer=%d, disconnecting\n", qb.hash.ToString().c_str(),
                      (int)pto->GetId());
            pto->fDisconnect = true;
            return true;
        }
    }

    // ---- block download
    std::vector<CInv> vGetData;
    if (!pto->fClient && (fFetch || !I.cs->IsInitialBlockDownload()) && st->nBlocksInFlight < MAX_BLOCKS_IN_TRANSIT_PER_PEER) {
        std::vector<const CBlockIndex*> vToDownload;
        NodeId staller = -1;
        I.FindNextBlocksToDownload(pto->GetId(), MAX_BLOCKS_IN_TRANSIT_PER_PEER - st->nBlocksInFlight, vToDownload, staller);
        for (const CBlockIndex* pi : vToDownload) {
            vGetData.push_back(CInv(MSG_BLOCK, pi->GetBlockHash()));
            I.MarkBlockAsInFlight(pto->GetId(), pi->GetBlockHash(), pi);
            LogPrint(BCLog::NET, "Requesting block %s (%d) peer=%d\n", pi->GetBlockHash().ToString().c_str(), pi->nHeight,
                     (int)pto->GetId());
        }
        if (st->nBlocksInFlight == 0 && staller != -1) {
            if (CNodeState* sst = I.State(staller))
                if (sst->nStallingSince == 0) {
                    sst->nStallingSince = nNow;
                    LogPrint(BCLog::NET, "Stall started peer=%d\n", (int)staller);
                }
        }
    }

    // ---- tx requests from AskFor
    {
        std::lock_guard<std::mutex> li(pto->cs_inventory);
        while (!pto->fDisconnect && !pto->mapAskFor.empty() && pto->mapAskFor.begin()->first <= nNow) {
            const CInv& inv = pto->mapAskFor.begin()->second;
            if (!I.AlreadyHave(inv)) {
                vGetData.push_back(inv);
                if (vGetData.size() >= 1000) {
                    I.Push(pto, msgMaker.Make(NetMsgType::GETDATA, vGetData));
                    vGetData.clear();
                }
            } else {
                // got it already: other peers need not be asked
                std::lock_guard<std::mutex> la(cs_mapAlreadyAskedFor);
                mapAlreadyAskedFor.erase(inv.hash);
            }
            pto->setAskFor.erase(inv.hash);
            pto->mapAskFor.erase(pto->mapAskFor.begin());
        }
    }
    if (!vGetData.empty()) I.Push(pto, msgMaker.Make(NetMsgType::GETDATA, vGetData));

    // ---- feefilter
    if (pto->nVersion >= FEEFILTER_VERSION && gArgs.GetBoolArg("-feefilter", true) &&
        !(pto->fWhitelisted && gArgs.GetBoolArg("-whitelistforcerelay", true))) {
        const int64_t maxmempool = gArgs.GetArg("-maxmempool", (int64_t)300) * 1000000;
        Amount currentFilter = I.pool->GetMinFee((size_t)maxmempool).GetFeePerK();
        const int64_t timeNow = GetTimeMicros();
        if (timeNow > pto->nextSendTimeFeeFilter) {
            static FeeFilterRounder filterRounder(minRelayTxFee);
            currentFilter = filterRounder.round(currentFilter);
            currentFilter = std::max(currentFilter, minRelayTxFee.GetFeePerK());
            if (currentFilter != pto->lastSentFeeFilter) {
                I.Push(pto, msgMaker.Make(NetMsgType::FEEFILTER, (int64_t)currentFilter));
                pto->lastSentFeeFilter = currentFilter;
            }
            pto->nextSendTimeFeeFilter = PoissonNextSend(timeNow, 10 * 60);
        }
    }
    (void)interrupt;
    return true;
}

} // namespace bcp
