#include "net/net.h"
#include "net/netbase.h"
#include "node/ui_interface.h"
#include "consensus/params.h"
#include "consensus/tx_verify.h"
#include "crypto/hashes.h"
#include "keys/key.h"
#include "util/strencodings.h"

#include <arpa/inet.h>
#include <cmath>
#include <fcntl.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <unistd.h>

namespace bcp {

std::atomic<bool> fListen{true};
std::atomic<bool> fDiscover{true};
static std::mutex cs_mapLocalHost;
static std::map<CNetAddr, std::pair<int, int>> mapLocalHost; // addr -> (port, score)
static CConnman* g_connman_ptr = nullptr;
CConnman* GetConnman() { return g_connman_ptr; }

// ------------------------------------------------------------------ local addresses
bool AddLocal(const CService& addr, int nScore) {
    if (!addr.IsRoutable()) return false;
    if (!fDiscover && nScore < LOCAL_MANUAL) return false;
    LogPrintf("AddLocal(%s,%i)\n", addr.ToString().c_str(), nScore);
    std::lock_guard<std::mutex> l(cs_mapLocalHost);
    auto it = mapLocalHost.find(addr);
    if (it == mapLocalHost.end() || nScore >= it->second.second)
        mapLocalHost[addr] = {addr.GetPort(), nScore + (it != mapLocalHost.end() ? 1 : 0)};
    return true;
}

bool RemoveLocal(const CService& addr) {
    std::lock_guard<std::mutex> l(cs_mapLocalHost);
    return mapLocalHost.erase(addr) > 0;
}

bool IsLocalAddr(const CService& addr) {
    std::lock_guard<std::mutex> l(cs_mapLocalHost);
    return mapLocalHost.count(addr) > 0;
}

bool GetLocal(CService& addr, const CNetAddr* paddrPeer) {
    if (!fListen) return false;
    int bestScore = -1;
    std::lock_guard<std::mutex> l(cs_mapLocalHost);
    for (const auto& kv : mapLocalHost) {
        if (paddrPeer && paddrPeer->GetNetwork() != NET_UNROUTABLE && kv.first.GetNetwork() != paddrPeer->GetNetwork() &&
            paddrPeer->IsIPv4() != kv.first.IsIPv4())
            continue;
        if (kv.second.second > bestScore) {
            addr = CService(kv.first, (uint16_t)kv.second.first);
            bestScore = kv.second.second;
        }
    }
    return bestScore >= 0;
}

CAddress GetLocalAddress(const CNetAddr* paddrPeer, uint64_t nLocalServices) {
    CAddress ret(CService(CNetAddr(), (uint16_t)Params().GetDefaultPort()), NODE_NONE);
    CService addr;
    if (GetLocal(addr, paddrPeer)) ret = CAddress(addr, nLocalServices);
    ret.nTime = (uint32_t)GetAdjustedTime();
    return ret;
}

std::map<CNetAddr, std::pair<int, int>> GetLocalAddresses() {
    std::lock_guard<std::mutex> l(cs_mapLocalHost);
    return mapLocalHost;
}

int64_t PoissonNextSend(int64_t nNow, int average_interval_seconds) {
    return nNow + (int64_t)(std::log1p(GetRand(1ULL << 48) * -0.0000000000000035527136788 /* -1/2^48 */) *
                                average_interval_seconds * -1000000.0 +
                            0.5);
}

// ------------------------------------------------------------------ CNode
CNode::CNode(NodeId idIn, uint64_t localServices, int startingHeight, int fd, const CAddress& addrIn,
             uint64_t keyedNetGroup, uint64_t localHostNonce, const std::string& name, bool inbound)
    : id(idIn), nTimeConnected(GetSystemTimeInSeconds()), addr(addrIn),
      addrName(name.empty() ? addrIn.ToStringIPPort() : name), fInbound(inbound), nKeyedNetGroup(keyedNetGroup),
      hSocket(fd), addrKnown(5000, 0.001), filterInventoryKnown(50000, 0.000001), nLocalHostNonce(localHostNonce),
      nLocalServices(localServices), nMyStartingHeight(startingHeight) {
    fRelayTxes = inbound ? false : true;
    for (const std::string& m : GetAllNetMessageTypes()) {
        mapRecvBytesPerMsgCmd[m] = 0;
        mapSendBytesPerMsgCmd[m] = 0;
    }
    mapRecvBytesPerMsgCmd["*other*"] = 0;
    LogPrint(BCLog::NET, "Added connection peer=%d\n", (int)id);
}

CNode::~CNode() { CloseSocketDisconnect(); }

void CNode::CloseSocketDisconnect() {
    fDisconnect = true;
    std::lock_guard<std::mutex> l(cs_hSocket);
    if (hSocket >= 0) {
        LogPrint(BCLog::NET, "disconnecting peer=%d\n", (int)id);
        close(hSocket);
        hSocket = -1;
    }
}

void CNode::SetAddrLocal(const CService& a) {
    std::lock_guard<std::mutex> l(cs_addrLocal);
    if (!addrLocal.IsValid()) addrLocal = a;
}
CService CNode::GetAddrLocal() const {
    std::lock_guard<std::mutex> l(cs_addrLocal);
    return addrLocal;
}

bool CNode::ReceiveMsgBytes(const unsigned char* p, size_t n, const unsigned char* magic, bool& complete) {
    complete = false;
    const int64_t now = GetTimeMicros();
    std::lock_guard<std::mutex> l(cs_vRecv);
    nLastRecv = now / 1000000;
    nRecvBytes += n;
    while (n > 0) {
        if (inHeader) {
            const size_t need = CMessageHeader::HEADER_SIZE - hdrbuf.size();
            const size_t take = std::min(need, n);
            hdrbuf.insert(hdrbuf.end(), p, p + take);
            p += take;
            n -= take;
            if (hdrbuf.size() < CMessageHeader::HEADER_SIZE) break;
            try {
                SpanReader r(hdrbuf.data(), hdrbuf.size());
                r >> curMsg.hdr;
            } catch (const std::exception&) {
                return false;
            }
            hdrbuf.clear();
            if (!curMsg.hdr.IsValid(magic)) {
                LogPrint(BCLog::NET, "invalid message header from peer=%d (%s)\n", (int)id,
                         SanitizeString(curMsg.hdr.GetCommand()).c_str());
                return false;
            }
            if (curMsg.hdr.nMessageSize > MAX_PROTOCOL_MESSAGE_LENGTH) return false;
            curMsg.payload.clear();
            curMsg.payload.reserve(std::min<size_t>(curMsg.hdr.nMessageSize, 256 * 1024));
            nDataPos = 0;
            inHeader = false;
        }
        if (!inHeader) {
            const size_t need = curMsg.hdr.nMessageSize - nDataPos;
            const size_t take = std::min(need, n);
            curMsg.payload.insert(curMsg.payload.end(), p, p + take);
            nDataPos += take;
            p += take;
            n -= take;
            if (nDataPos == curMsg.hdr.nMessageSize) {
                curMsg.nTime = now;
                unsigned char sum[4];
                MessageChecksum(curMsg.payload.data(), curMsg.payload.size(), sum);
                const std::string cmd = curMsg.hdr.GetCommand();
                auto it = mapRecvBytesPerMsgCmd.find(cmd);
                if (it == mapRecvBytesPerMsgCmd.end()) it = mapRecvBytesPerMsgCmd.find("*other*");
                it->second += curMsg.payload.size() + CMessageHeader::HEADER_SIZE;
                if (memcmp(sum, curMsg.hdr.checksum.data(), 4) != 0) {
                    LogPrint(BCLog::NET, "CHECKSUM ERROR (%s, %u bytes) peer=%d\n", SanitizeString(cmd).c_str(),
                             curMsg.hdr.nMessageSize, (int)id);
                    // the reference drops the message but keeps the peer
                } else {
                    completed.push_back(std::move(curMsg));
                    complete = true;
                }
                curMsg = CNetMessage();
                inHeader = true;
            }
        }
    }
    return true;
}

void CNode::AddAddressKnown(const CAddress& a) { addrKnown.insert(a.GetKey()); }

void CNode::PushAddress(const CAddress& a, FastRandomContext& rng) {
    // known addresses are skipped; a full buffer replaces a random slot
    if (a.IsValid() && !addrKnown.contains(a.GetKey())) {
        if (vAddrToSend.size() >= MAX_ADDR_TO_SEND)
            vAddrToSend[rng.randrange(vAddrToSend.size())] = a;
        else
            vAddrToSend.push_back(a);
    }
}

void CNode::AddInventoryKnown(const CInv& inv) {
    std::lock_guard<std::mutex> l(cs_inventory);
    filterInventoryKnown.insert(inv.hash);
}

void CNode::PushInventory(const CInv& inv) {
    std::lock_guard<std::mutex> l(cs_inventory);
    if (inv.type == MSG_TX) {
        if (!filterInventoryKnown.contains(inv.hash)) setInventoryTxToSend.insert(inv.hash);
    } else if (inv.type == MSG_BLOCK) {
        vInventoryBlockToSend.push_back(inv.hash);
    }
}

void CNode::PushBlockHash(const uint256& hash) {
    std::lock_guard<std::mutex> l(cs_inventory);
    vBlockHashesToAnnounce.push_back(hash);
}

limitedmap<uint256, int64_t> mapAlreadyAskedFor(MAX_INV_SZ);
std::mutex cs_mapAlreadyAskedFor;

void CNode::AskFor(const CInv& inv) {
    std::lock_guard<std::mutex> l(cs_inventory);
    if (mapAskFor.size() > MAX_INV_SZ || setAskFor.size() > MAX_INV_SZ) return;
    if (!setAskFor.insert(inv.hash).second) return; // already queued from this peer
    // each further peer asked for the same hash waits 2 minutes longer, so one slow or lying
    // peer delays but never blocks relay; request times are kept strictly increasing
    static int64_t nLastTime = 0;
    std::lock_guard<std::mutex> la(cs_mapAlreadyAskedFor);
    int64_t nNow = GetTimeMicros() - 1000000;
    nNow = std::max(nNow, ++nLastTime);
    nLastTime = nNow;
    auto it = mapAlreadyAskedFor.find(inv.hash);
    const int64_t nRequestTime = std::max(it != mapAlreadyAskedFor.end() ? it->second + 2 * 60 * 1000000 : 0, nNow);
    if (it != mapAlreadyAskedFor.end()) mapAlreadyAskedFor.update(it, nRequestTime);
    else mapAlreadyAskedFor.insert({inv.hash, nRequestTime});
    mapAskFor.insert({nRequestTime, inv});
}

void CNode::CopyStats(CNodeStats& st) const {
    st.nodeid = id;
    st.nServices = nServices;
    st.addr = addr;
    {
        std::lock_guard<std::mutex> l(const_cast<std::mutex&>(cs_filter));
        st.fRelayTxes = fRelayTxes;
    }
    st.nLastSend = nLastSend;
    st.nLastRecv = nLastRecv;
    st.nTimeConnected = nTimeConnected;
    st.nTimeOffset = nTimeOffset;
    st.addrName = addrName;
    st.nVersion = nVersion;
    {
        std::lock_guard<std::mutex> l(const_cast<std::mutex&>(cs_SubVer));
        st.cleanSubVer = cleanSubVer;
    }
    st.fInbound = fInbound;
    st.fAddnode = fAddnode;
    st.fWhitelisted = fWhitelisted;
    st.nStartingHeight = nStartingHeight;
    st.nSendBytes = nSendBytes;
    st.nRecvBytes = nRecvBytes;
    {
        std::lock_guard<std::mutex> l(const_cast<std::mutex&>(cs_vSend));
        st.mapSendBytesPerMsgCmd = mapSendBytesPerMsgCmd;
    }
    {
        std::lock_guard<std::mutex> l(const_cast<std::mutex&>(cs_vRecv));
        st.mapRecvBytesPerMsgCmd = mapRecvBytesPerMsgCmd;
    }
    const int64_t pingStart = nPingUsecStart;
    st.dPingTime = nPingUsecTime * 1e-6;
    st.dMinPing = nMinPingUsecTime == INT64_MAX ? 0 : nMinPingUsecTime * 1e-6;
    st.dPingWait = (nPingNonceSent && pingStart) ? (GetTimeMicros() - pingStart) * 1e-6 : 0;
    const CService local = GetAddrLocal();
    st.addrLocal = local.IsValid() ? local.ToString() : "";
}

// ------------------------------------------------------------------ CConnman
CConnman::CConnman(uint64_t seed0, uint64_t seed1) : nSeed0(seed0), nSeed1(seed1) {}

CConnman::~CConnman() {
    Interrupt();
    Stop();
}

CSipHasher CConnman::GetDeterministicRandomizer(uint64_t id) const { return CSipHasher(nSeed0, nSeed1).Write(id); }

static void SetNonBlocking(int fd) {
    const int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags | O_NONBLOCK);
}

bool CConnman::BindListenPort(const CService& bind, std::string& err, bool fWhitelisted) {
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (!bind.GetSockAddr((struct sockaddr*)&ss, &len)) {
        err = "Error: Bind address family for " + bind.ToString() + " not supported";
        return false;
    }
    const int fd = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
    if (fd < 0) {
        err = "Error: Couldn't open socket for incoming connections";
        return false;
    }
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (!bind.IsIPv4()) setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &one, sizeof(one));
    SetNonBlocking(fd);
    if (::bind(fd, (struct sockaddr*)&ss, len) != 0) {
        err = strprintf("Unable to bind to %s on this computer (%s)", bind.ToString().c_str(), strerror(errno));
        close(fd);
        return false;
    }
    if (listen(fd, SOMAXCONN) != 0) {
        err = strprintf("Error: Listening for incoming connections failed (%s)", strerror(errno));
        close(fd);
        return false;
    }
    LogPrintf("Bound to %s\n", bind.ToString().c_str());
    vhListenSocket.push_back({fd, fWhitelisted});
    if (bind.IsRoutable() && fDiscover && !fWhitelisted) AddLocal(bind, LOCAL_BIND);
    return true;
}

bool CConnman::Start(Scheduler* scheduler, const Options& o, std::string& err) {
    nLocalServices = o.nLocalServices;
    nRelevantServices = o.nRelevantServices;
    nMaxConnections = o.nMaxConnections;
    nMaxOutbound = std::min(o.nMaxOutbound, o.nMaxConnections);
    nMaxAddnode = o.nMaxAddnode;
    nMaxFeeler = o.nMaxFeeler;
    nBestHeight = o.nBestHeight;
    events = o.events;
    nSendBufferMaxSize = o.nSendBufferMaxSize;
    nReceiveFloodSize = o.nReceiveFloodSize;
    {
        std::lock_guard<Mutex> l(cs_totalBytesSent);
        nMaxOutboundLimit = o.nMaxOutboundLimit;
        nMaxOutboundTimeframe = o.nMaxOutboundTimeframe;
    }
    vWhitelistedRange = o.vWhitelistedRange;
    vConnect = o.vConnect;
    fConnectOnly = o.fConnectOnly;
    fDNSSeed = o.fDNSSeed;
    fForceDNSSeed = o.fForceDNSSeed;
    datadir = o.datadir;
    {
        std::lock_guard<Mutex> l(cs_vOneShots);
        for (const std::string& s : o.vSeedNodes) vOneShots.push_back(s);
    }

    if (!datadir.empty()) {
        if (addrman.Read(datadir + "/peers.dat", Params().NetMagic()))
            LogPrintf("Loaded %zu addresses from peers.dat\n", addrman.size());
        else
            LogPrintf("Invalid or missing peers.dat; recreating\n");
        if (banman.Read(datadir + "/banlist.dat", Params().NetMagic())) {
            banmap_t m;
            banman.GetBanned(m);
            LogPrintf("Loaded %zu banned node ips/subnets from banlist.dat\n", m.size());
        }
    }
    if (o.fListen) {
        bool bound = false;
        for (const CService& b : o.vBinds) {
            std::string e;
            if (BindListenPort(b, e, false)) {
                bound = true;
                nListenPort = b.GetPort();
            } else if (!o.fDefaultBinds) {
                err = e;
                return false;
            } else {
                LogPrintf("%s\n", e.c_str());
                if (err.empty()) err = e;
            }
        }
        for (const CService& b : o.vWhiteBinds) {
            std::string e;
            if (!BindListenPort(b, e, true)) {
                err = e;
                return false;
            }
            bound = true;
        }
        if (!bound) {
            err = "Failed to listen on any port. " + err;
            return false;
        }
        err.clear();
    }
    if (pipe(wakeupPipe) != 0) {
        err = "pipe() failed";
        return false;
    }
    SetNonBlocking(wakeupPipe[0]);
    SetNonBlocking(wakeupPipe[1]);
    interruptNet = false;
    flagInterruptMsgProc = false;
    g_connman_ptr = this;

    threadSocketHandler = std::thread([this] { RenameThread("bcp-net"); ThreadSocketHandler(); });
    if (fDNSSeed && !fConnectOnly && !Params().DNSSeeds().empty())
        threadDNSAddressSeed = std::thread([this] { RenameThread("bcp-dnsseed"); ThreadDNSAddressSeed(); });
    threadOpenAddedConnections = std::thread([this] { RenameThread("bcp-addcon"); ThreadOpenAddedConnections(); });
    threadOpenConnections = std::thread([this] { RenameThread("bcp-opencon"); ThreadOpenConnections(); });
    threadMessageHandler = std::thread([this] { RenameThread("bcp-msghand"); ThreadMessageHandler(); });
    if (scheduler) scheduler->ScheduleEvery([this] { DumpData(); }, DUMP_ADDRESSES_INTERVAL * 1000);
    started = true;
    return true;
}

void CConnman::Interrupt() {
    {
        std::lock_guard<std::mutex> l(mutexMsgProc);
        flagInterruptMsgProc = true;
    }
    condMsgProc.notify_all();
    interruptNet = true;
    cv_sleep.notify_all();
    if (wakeupPipe[1] >= 0) {
        char c = 0;
        (void)!write(wakeupPipe[1], &c, 1);
    }
}

void CConnman::Stop() {
    if (!started) return;
    Interrupt();
    if (threadMessageHandler.joinable()) threadMessageHandler.join();
    if (threadOpenConnections.joinable()) threadOpenConnections.join();
    if (threadOpenAddedConnections.joinable()) threadOpenAddedConnections.join();
    if (threadDNSAddressSeed.joinable()) threadDNSAddressSeed.join();
    if (threadSocketHandler.joinable()) threadSocketHandler.join();
    DumpData();
    std::vector<CNode*> nodes;
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        nodes = vNodes;
        vNodes.clear();
    }
    for (CNode* p : nodes) {
        p->CloseSocketDisconnect();
        bool fUpdate = false;
        if (events) events->FinalizeNode(p->GetId(), fUpdate);
        delete p;
    }
    for (CNode* p : vNodesDisconnected) delete p;
    vNodesDisconnected.clear();
    for (const ListenSocket& ls : vhListenSocket) close(ls.fd);
    vhListenSocket.clear();
    if (wakeupPipe[0] >= 0) close(wakeupPipe[0]);
    if (wakeupPipe[1] >= 0) close(wakeupPipe[1]);
    wakeupPipe[0] = wakeupPipe[1] = -1;
    if (g_connman_ptr == this) g_connman_ptr = nullptr;
    started = false;
}

void CConnman::DumpData() {
    if (datadir.empty()) return;
    const int64_t t0 = GetTimeMillis();
    addrman.Write(datadir + "/peers.dat", Params().NetMagic());
    banman.Write(datadir + "/banlist.dat", Params().NetMagic());
    LogPrint(BCLog::NET, "Flushed %zu addresses to peers.dat  %dms\n", addrman.size(), (int)(GetTimeMillis() - t0));
}

void CConnman::SetNetworkActive(bool active) {
    LogPrintf("SetNetworkActive: %s\n", active ? "true" : "false");
    if (fNetworkActive == active) return;
    fNetworkActive = active;
    uiInterface.NotifyNetworkActiveChanged(active);
    if (!active) {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        for (CNode* p : vNodes) p->fDisconnect = true;
    }
}

bool CConnman::IsWhitelistedRange(const CNetAddr& addr) {
    for (const CSubNet& s : vWhitelistedRange)
        if (s.Match(addr)) return true;
    return false;
}

CNode* CConnman::FindNode(const CNetAddr& ip) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if ((CNetAddr)p->addr == ip) return p;
    return nullptr;
}
CNode* CConnman::FindNode(const std::string& name) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (p->addrName == name) return p;
    return nullptr;
}
CNode* CConnman::FindNode(const CService& addr) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if ((CService)p->addr == addr) return p;
    return nullptr;
}

bool CConnman::CheckIncomingNonce(uint64_t nonce) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (!p->fSuccessfullyConnected && !p->fInbound && p->GetLocalNonce() == nonce) return false;
    return true;
}

CNode* CConnman::ConnectNode(CAddress addrConnect, const char* pszDest) {
    if (pszDest == nullptr) {
        if (IsLocalAddr(addrConnect)) return nullptr;
        if (CNode* p = FindNode((CService)addrConnect)) {
            (void)p;
            LogPrintf("Failed to open new connection, already connected\n");
            return nullptr;
        }
    }
    LogPrint(BCLog::NET, "trying connection %s lastseen=%.1fhrs\n", pszDest ? pszDest : addrConnect.ToString().c_str(),
             pszDest ? 0.0 : (double)(GetAdjustedTime() - addrConnect.nTime) / 3600.0);
    const int timeoutMs = (int)gArgs.GetArg("-timeout", (int64_t)5000);
    int fd = -1;
    bool proxyConnectionFailed = false;
    proxyType nameProxy;
    if (pszDest && GetNameProxy(nameProxy)) {
        // -proxy set: hand the name to the proxy, never resolve it locally
        int port = Params().GetDefaultPort();
        std::string host;
        SplitHostPort(pszDest, port, host);
        fd = ConnectThroughProxy(nameProxy, host, (uint16_t)port, timeoutMs, &proxyConnectionFailed);
        if (fd >= 0) {
            CService svc = LookupNumeric(host, port);
            if (!svc.IsValid()) svc = nameProxy.proxy; // the peer's address stays unknown to us
            addrConnect = CAddress(svc, NODE_NONE);
        }
    } else {
        if (pszDest) {
            std::vector<CService> resolved;
            if (Lookup(pszDest, resolved, Params().GetDefaultPort(), fNameLookup, 256) && !resolved.empty()) {
                addrConnect = CAddress(resolved[GetRand(resolved.size())], NODE_NONE);
                if (!addrConnect.IsValid()) return nullptr;
                std::lock_guard<CCriticalSection> l(cs_vNodes);
                if (FindNode((CService)addrConnect)) {
                    LogPrintf("Failed to open new connection, already connected\n");
                    return nullptr;
                }
            } else {
                return nullptr;
            }
        }
        if (!IsReachable(addrConnect)) return nullptr; // -onlynet excludes this network
        proxyType proxy;
        if (GetProxy(addrConnect.GetNetwork(), proxy))
            fd = ConnectThroughProxy(proxy, addrConnect.ToStringIP(), addrConnect.GetPort(), timeoutMs,
                                     &proxyConnectionFailed);
        else if (!addrConnect.IsTor()) // onion peers are only reachable through a proxy
            fd = ConnectDirectly(addrConnect, timeoutMs);
    }
    if (fd < 0) {
        // a dead proxy says nothing about the peer: do not count it as a failed attempt
        if (!proxyConnectionFailed && !pszDest) addrman.Attempt(addrConnect, true);
        return nullptr;
    }
    addrman.Attempt(addrConnect, false);
    const NodeId id = nLastNodeId++;
    const uint64_t nonce = GetDeterministicRandomizer(0xd93e69e2bbfa5735ULL).Write(id).Finalize();
    const std::vector<unsigned char> grp = addrConnect.GetGroup();
    const uint64_t keyed = GetDeterministicRandomizer(0x6c0edd8036ef4036ULL).Write(grp.data(), grp.size()).Finalize();
    CNode* p = new CNode(id, nLocalServices, nBestHeight, fd, addrConnect, keyed, nonce, pszDest ? pszDest : "", false);
    p->nServices = addrConnect.nServices;
    p->AddRef();
    return p;
}

bool CConnman::OpenNetworkConnection(const CAddress& addrConnect, bool fCountFailure, const char* pszDest,
                                     bool fOneShot, bool fFeeler, bool fAddnode) {
    if (interruptNet || !fNetworkActive) return false;
    if (!pszDest) {
        if (IsLocalAddr(addrConnect) || FindNode((CNetAddr)addrConnect) || IsBanned(addrConnect) ||
            FindNode(addrConnect.ToStringIPPort()))
            return false;
    } else if (FindNode(std::string(pszDest))) {
        return false;
    }
    CNode* p = ConnectNode(addrConnect, pszDest);
    (void)fCountFailure;
    if (!p) return false;
    p->fOneShot = fOneShot;
    p->fFeeler = fFeeler;
    p->fAddnode = fAddnode;
    if (events) events->InitializeNode(p);
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        vNodes.push_back(p);
    }
    WakeMessageHandler();
    return true;
}

bool CConnman::AttemptToEvictConnection() {
    // Protect peers by several independent criteria, then evict the youngest member of
    // the largest remaining netgroup (reference net.cpp:872-990 simplified to its core).
    struct Cand {
        NodeId id;
        int64_t connected, minPing;
        uint64_t keyedGroup;
    };
    std::vector<Cand> cands;
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        for (CNode* p : vNodes) {
            if (p->fWhitelisted || !p->fInbound || p->fDisconnect) continue;
            cands.push_back({p->GetId(), p->nTimeConnected, p->nMinPingUsecTime, p->nKeyedNetGroup});
        }
    }
    if (cands.empty()) return false;
    auto protect = [&](auto cmp, size_t n) {
        std::sort(cands.begin(), cands.end(), cmp);
        cands.erase(cands.end() - std::min(n, cands.size()), cands.end());
    };
    protect([](const Cand& a, const Cand& b) { return a.keyedGroup > b.keyedGroup; }, 4);  // distinct groups
    protect([](const Cand& a, const Cand& b) { return a.minPing > b.minPing; }, 8);         // lowest ping
    protect([](const Cand& a, const Cand& b) { return a.connected > b.connected; }, cands.size() / 2); // oldest half
    if (cands.empty()) return false;
    std::map<uint64_t, std::vector<Cand>> groups;
    for (const Cand& c : cands) groups[c.keyedGroup].push_back(c);
    const std::vector<Cand>* worst = nullptr;
    for (const auto& kv : groups)
        if (!worst || kv.second.size() > worst->size()) worst = &kv.second;
    const Cand* youngest = nullptr;
    for (const Cand& c : *worst)
        if (!youngest || c.connected > youngest->connected) youngest = &c;
    return DisconnectNode(youngest->id);
}

void CConnman::AcceptConnection(const ListenSocket& ls) {
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    const int fd = accept(ls.fd, (struct sockaddr*)&ss, &len);
    if (fd < 0) return;
    CAddress addr;
    CService svc;
    if (svc.SetSockAddr((struct sockaddr*)&ss)) addr = CAddress(svc, NODE_NONE);
    const bool whitelisted = ls.whitelisted || IsWhitelistedRange(addr);
    int nInbound = 0;
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        for (CNode* p : vNodes)
            if (p->fInbound) nInbound++;
    }
    if (!fNetworkActive) {
        LogPrintf("connection from %s dropped: not accepting new connections\n", addr.ToString().c_str());
        close(fd);
        return;
    }
    if (IsBanned(addr) && !whitelisted) {
        LogPrint(BCLog::NET, "connection from %s dropped (banned)\n", addr.ToString().c_str());
        close(fd);
        return;
    }
    const int nMaxInbound = nMaxConnections - (nMaxOutbound + nMaxFeeler);
    if (nInbound >= nMaxInbound) {
        if (!AttemptToEvictConnection()) {
            LogPrint(BCLog::NET, "failed to find an eviction candidate - connection dropped (full)\n");
            close(fd);
            return;
        }
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    SetNonBlocking(fd);
    const NodeId id = nLastNodeId++;
    const uint64_t nonce = GetDeterministicRandomizer(0xd93e69e2bbfa5735ULL).Write(id).Finalize();
    const std::vector<unsigned char> grp = addr.GetGroup();
    const uint64_t keyed = GetDeterministicRandomizer(0x6c0edd8036ef4036ULL).Write(grp.data(), grp.size()).Finalize();
    CNode* p = new CNode(id, nLocalServices, nBestHeight, fd, addr, keyed, nonce, "", true);
    p->AddRef();
    p->fWhitelisted = whitelisted;
    if (events) events->InitializeNode(p);
    LogPrint(BCLog::NET, "connection from %s accepted\n", addr.ToString().c_str());
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        vNodes.push_back(p);
    }
}

void CConnman::RecordBytesSent(uint64_t n) {
    nTotalBytesSent += n;
    std::lock_guard<Mutex> l(cs_totalBytesSent);
    const uint64_t now = GetTime();
    if (nMaxOutboundCycleStartTime + nMaxOutboundTimeframe < now) {
        nMaxOutboundCycleStartTime = now;
        nMaxOutboundTotalBytesSentInCycle = 0;
    }
    nMaxOutboundTotalBytesSentInCycle += n;
}

bool CConnman::OutboundTargetReached(bool historicalBlockServingLimit) {
    std::lock_guard<Mutex> l(cs_totalBytesSent);
    if (nMaxOutboundLimit == 0) return false;
    if (historicalBlockServingLimit) {
        const uint64_t timeLeft = nMaxOutboundCycleStartTime + nMaxOutboundTimeframe - (uint64_t)GetTime();
        const uint64_t buffer = timeLeft / 600 * DEFAULT_MAX_BLOCK_SIZE;
        if (buffer >= nMaxOutboundLimit || nMaxOutboundTotalBytesSentInCycle >= nMaxOutboundLimit - buffer) return true;
    } else if (nMaxOutboundTotalBytesSentInCycle >= nMaxOutboundLimit) {
        return true;
    }
    return false;
}

uint64_t CConnman::GetOutboundTargetBytesLeft() {
    std::lock_guard<Mutex> l(cs_totalBytesSent);
    if (nMaxOutboundLimit == 0) return 0;
    return nMaxOutboundTotalBytesSentInCycle >= nMaxOutboundLimit ? 0
                                                                   : nMaxOutboundLimit - nMaxOutboundTotalBytesSentInCycle;
}

uint64_t CConnman::GetMaxOutboundTimeLeftInCycle() {
    std::lock_guard<Mutex> l(cs_totalBytesSent);
    if (nMaxOutboundLimit == 0) return 0;
    if (nMaxOutboundCycleStartTime == 0) return nMaxOutboundTimeframe;
    const uint64_t end = nMaxOutboundCycleStartTime + nMaxOutboundTimeframe;
    const uint64_t now = GetTime();
    return end < now ? 0 : end - now;
}

void CConnman::SocketSendData(CNode* p) {
    // caller holds p->cs_vSend
    while (!p->vSendMsg.empty()) {
        const std::vector<unsigned char>& d = p->vSendMsg.front();
        int n;
        {
            std::lock_guard<std::mutex> l(p->cs_hSocket);
            if (p->hSocket < 0) break;
            n = (int)send(p->hSocket, d.data() + p->nSendOffset, d.size() - p->nSendOffset, MSG_NOSIGNAL | MSG_DONTWAIT);
        }
        if (n > 0) {
            p->nLastSend = GetSystemTimeInSeconds();
            p->nSendBytes += n;
            p->nSendOffset += n;
            RecordBytesSent(n);
            if (p->nSendOffset == d.size()) {
                p->nSendOffset = 0;
                p->nSendSize -= d.size();
                p->fPauseSend = p->nSendSize > nSendBufferMaxSize;
                p->vSendMsg.pop_front();
            } else {
                break; // could not send the whole buffer
            }
        } else {
            if (n < 0 && errno != EWOULDBLOCK && errno != EAGAIN && errno != EINTR) {
                LogPrint(BCLog::NET, "socket send error peer=%d: %s\n", (int)p->GetId(), strerror(errno));
                p->CloseSocketDisconnect();
            }
            break;
        }
    }
}

void CConnman::PushMessage(CNode* p, CSerializedNetMsg&& msg) {
    const size_t nMessageSize = msg.data.size();
    LogPrint(BCLog::NET, "sending %s (%zu bytes) peer=%d\n", SanitizeString(msg.command).c_str(), nMessageSize,
             (int)p->GetId());
    CMessageHeader hdr(Params().NetMagic(), msg.command.c_str(), (uint32_t)nMessageSize);
    MessageChecksum(msg.data.data(), msg.data.size(), hdr.checksum.data());
    std::vector<unsigned char> wire;
    wire.reserve(CMessageHeader::HEADER_SIZE + nMessageSize);
    {
        VectorWriter w(wire);
        w << hdr;
    }
    wire.insert(wire.end(), msg.data.begin(), msg.data.end());
    std::lock_guard<std::mutex> l(p->cs_vSend);
    const bool optimistic = p->vSendMsg.empty();
    auto it = p->mapSendBytesPerMsgCmd.find(msg.command);
    if (it != p->mapSendBytesPerMsgCmd.end()) it->second += wire.size();
    p->nSendSize += wire.size();
    if (p->nSendSize > nSendBufferMaxSize) p->fPauseSend = true;
    p->vSendMsg.push_back(std::move(wire));
    if (optimistic) SocketSendData(p);
    else if (wakeupPipe[1] >= 0) {
        char c = 1;
        (void)!write(wakeupPipe[1], &c, 1);
    }
}

void CConnman::ThreadSocketHandler() {
    size_t nPrevNodeCount = 0;
    std::vector<unsigned char> buf(0x10000);
    while (!interruptNet) {
        // ---- disconnect and reap nodes
        {
            std::lock_guard<CCriticalSection> l(cs_vNodes);
            std::vector<CNode*> copy = vNodes;
            for (CNode* p : copy) {
                if (p->fDisconnect) {
                    vNodes.erase(std::remove(vNodes.begin(), vNodes.end(), p), vNodes.end());
                    p->CloseSocketDisconnect();
                    p->Release();
                    vNodesDisconnected.push_back(p);
                }
            }
        }
        for (auto it = vNodesDisconnected.begin(); it != vNodesDisconnected.end();) {
            CNode* p = *it;
            if (p->GetRefCount() <= 0) {
                bool fUpdate = false;
                if (events) events->FinalizeNode(p->GetId(), fUpdate);
                if (fUpdate) addrman.Connected(p->addr);
                it = vNodesDisconnected.erase(it);
                delete p;
            } else {
                ++it;
            }
        }
        size_t n;
        {
            std::lock_guard<CCriticalSection> l(cs_vNodes);
            n = vNodes.size();
        }
        if (n != nPrevNodeCount) {
            nPrevNodeCount = n;
            uiInterface.NotifyNumConnectionsChanged((int)n);
        }

        // ---- poll
        std::vector<struct pollfd> fds;
        std::vector<CNode*> pollNodes;
        fds.push_back({wakeupPipe[0], POLLIN, 0});
        for (const ListenSocket& ls : vhListenSocket) fds.push_back({ls.fd, POLLIN, 0});
        const size_t nodeBase = fds.size();
        {
            std::lock_guard<CCriticalSection> l(cs_vNodes);
            for (CNode* p : vNodes) {
                short ev = 0;
                {
                    std::lock_guard<std::mutex> ls(p->cs_vSend);
                    if (!p->vSendMsg.empty()) ev |= POLLOUT;
                }
                if (!p->fPauseRecv) ev |= POLLIN;
                int fd;
                {
                    std::lock_guard<std::mutex> lh(p->cs_hSocket);
                    fd = p->hSocket;
                }
                if (fd < 0) continue;
                fds.push_back({fd, ev, 0});
                pollNodes.push_back(p->AddRef());
            }
        }
        const int rc = poll(fds.data(), fds.size(), 50);
        if (interruptNet) {
            for (CNode* p : pollNodes) p->Release();
            break;
        }
        if (rc > 0) {
            if (fds[0].revents & POLLIN) {
                char tmp[64];
                while (read(wakeupPipe[0], tmp, sizeof(tmp)) > 0) {
                }
            }
            for (size_t i = 0; i < vhListenSocket.size(); i++)
                if (fds[1 + i].revents & POLLIN) AcceptConnection(vhListenSocket[i]);
            for (size_t i = 0; i < pollNodes.size(); i++) {
                CNode* p = pollNodes[i];
                const short re = fds[nodeBase + i].revents;
                if (re & (POLLIN | POLLERR | POLLHUP)) {
                    ssize_t got;
                    {
                        std::lock_guard<std::mutex> l(p->cs_hSocket);
                        if (p->hSocket < 0) continue;
                        got = recv(p->hSocket, buf.data(), buf.size(), MSG_DONTWAIT);
                    }
                    if (got > 0) {
                        bool complete = false;
                        if (!p->ReceiveMsgBytes(buf.data(), (size_t)got, Params().NetMagic(), complete)) {
                            p->CloseSocketDisconnect();
                        }
                        nTotalBytesRecv += got;
                        if (complete) {
                            size_t sz = 0;
                            std::vector<CNetMessage> msgs;
                            {
                                std::lock_guard<std::mutex> l(p->cs_vRecv);
                                msgs.swap(p->completed);
                            }
                            for (const CNetMessage& m : msgs) sz += m.payload.size() + CMessageHeader::HEADER_SIZE;
                            {
                                std::lock_guard<std::mutex> l(p->cs_vProcessMsg);
                                for (CNetMessage& m : msgs) p->vProcessMsg.push_back(std::move(m));
                                p->nProcessQueueSize += sz;
                                p->fPauseRecv = p->nProcessQueueSize > nReceiveFloodSize;
                            }
                            WakeMessageHandler();
                        }
                    } else if (got == 0) {
                        if (!p->fDisconnect) LogPrint(BCLog::NET, "socket closed for peer=%d\n", (int)p->GetId());
                        p->CloseSocketDisconnect();
                    } else if (errno != EWOULDBLOCK && errno != EAGAIN && errno != EINTR) {
                        if (!p->fDisconnect) LogPrint(BCLog::NET, "socket recv error peer=%d: %s\n", (int)p->GetId(), strerror(errno));
                        p->CloseSocketDisconnect();
                    }
                }
                if (re & POLLOUT) {
                    std::lock_guard<std::mutex> l(p->cs_vSend);
                    SocketSendData(p);
                }
            }
        }
        // ---- inactivity checks
        const int64_t now = GetSystemTimeInSeconds();
        // -peertimeout: the window a new connection has to exchange its first messages and
        // finish the version handshake (60 s as in the reference); after that, the 20-minute
        // send/receive/ping timeouts apply
        const int64_t connectWindow = std::max<int64_t>(1, gArgs.GetArg("-peertimeout", (int64_t)60));
        const int64_t timeout = TIMEOUT_INTERVAL;
        for (CNode* p : pollNodes) {
            if (now - p->nTimeConnected > connectWindow) {
                if (p->nLastRecv == 0 || p->nLastSend == 0) {
                    LogPrint(BCLog::NET, "socket no message in first %d seconds, %d %d from %d\n", (int)connectWindow,
                             p->nLastRecv != 0, p->nLastSend != 0, (int)p->GetId());
                    p->fDisconnect = true;
                } else if (now - p->nLastSend > timeout) {
                    LogPrintf("socket sending timeout: %ds\n", (int)(now - p->nLastSend));
                    p->fDisconnect = true;
                } else if (now - p->nLastRecv > (p->nVersion > BIP0031_VERSION ? timeout : 90 * 60)) {
                    LogPrintf("socket receive timeout: %ds\n", (int)(now - p->nLastRecv));
                    p->fDisconnect = true;
                } else if (p->nPingNonceSent && p->nPingUsecStart + timeout * 1000000 < GetTimeMicros()) {
                    LogPrintf("ping timeout: %fs\n", 0.000001 * (GetTimeMicros() - p->nPingUsecStart));
                    p->fDisconnect = true;
                } else if (!p->fSuccessfullyConnected) {
                    LogPrint(BCLog::NET, "version handshake timeout from %d\n", (int)p->GetId());
                    p->fDisconnect = true;
                }
            }
            p->Release();
        }
    }
}

void CConnman::WakeMessageHandler() {
    {
        std::lock_guard<std::mutex> l(mutexMsgProc);
        fMsgProcWake = true;
    }
    condMsgProc.notify_one();
}

void CConnman::ThreadMessageHandler() {
    while (!flagInterruptMsgProc) {
        std::vector<CNode*> copy;
        {
            std::lock_guard<CCriticalSection> l(cs_vNodes);
            for (CNode* p : vNodes) copy.push_back(p->AddRef());
        }
        bool fMoreWork = false;
        for (CNode* p : copy) {
            if (p->fDisconnect) continue;
            if (events) {
                const bool more = events->ProcessMessages(p, flagInterruptMsgProc);
                fMoreWork |= more && !p->fPauseSend;
                if (flagInterruptMsgProc) break;
                events->SendMessages(p, flagInterruptMsgProc);
            }
            if (flagInterruptMsgProc) break;
        }
        for (CNode* p : copy) p->Release();
        std::unique_lock<std::mutex> l(mutexMsgProc);
        if (!fMoreWork)
            condMsgProc.wait_for(l, std::chrono::milliseconds(100), [this] { return fMsgProcWake || flagInterruptMsgProc.load(); });
        fMsgProcWake = false;
    }
}

bool CConnman::InterruptibleSleep(int64_t millis) {
    std::unique_lock<std::mutex> l(cs_sleep);
    cv_sleep.wait_for(l, std::chrono::milliseconds(millis), [this] { return interruptNet.load(); });
    return !interruptNet;
}

void CConnman::ProcessOneShot() {
    std::string dest;
    {
        std::lock_guard<Mutex> l(cs_vOneShots);
        if (vOneShots.empty()) return;
        dest = vOneShots.front();
        vOneShots.pop_front();
    }
    CAddress addr;
    if (!OpenNetworkConnection(addr, false, dest.c_str(), true)) {
        std::lock_guard<Mutex> l(cs_vOneShots);
        vOneShots.push_back(dest);
    }
}

void CConnman::ThreadOpenConnections() {
    if (fConnectOnly) {
        for (int64_t loop = 0; !interruptNet; loop++) {
            ProcessOneShot();
            for (const std::string& s : vConnect) {
                CAddress addr;
                OpenNetworkConnection(addr, false, s.c_str());
                for (int i = 0; i < 10 && i < loop; i++)
                    if (!InterruptibleSleep(500)) return;
            }
            if (!InterruptibleSleep(500)) return;
        }
        return;
    }
    int64_t nStart = GetTime();
    int64_t nNextFeeler = PoissonNextSend(nStart * 1000 * 1000, FEELER_INTERVAL);
    while (!interruptNet) {
        ProcessOneShot();
        if (!InterruptibleSleep(500)) return;
        if (!fNetworkActive) continue;
        // regtest never auto-connects
        if (Params().MineBlocksOnDemand()) continue;
        // no addresses a minute after start (DNS seeds unreachable or disabled): fall back to the
        // compiled-in fixed seeds once (reference net.cpp ThreadOpenConnections)
        if (addrman.size() == 0 && GetTime() - nStart > 60 && !fFixedSeedsAdded) {
            fFixedSeedsAdded = true;
            const std::vector<CAddress> seeds = ConvertSeed6(Params().FixedSeeds());
            if (!seeds.empty()) {
                LogPrintf("Adding %u fixed seed nodes as DNS doesn't seem to be available.\n", (unsigned)seeds.size());
                CNetAddr local;
                local.SetIPv4(0x7f000001);
                addrman.Add(seeds, CAddress(CService(local, 0), NODE_NONE));
            }
        }
        int nOutbound = 0;
        std::set<std::vector<unsigned char>> setConnected;
        {
            std::lock_guard<CCriticalSection> l(cs_vNodes);
            for (CNode* p : vNodes)
                if (!p->fInbound && !p->fAddnode) {
                    setConnected.insert(p->addr.GetGroup());
                    nOutbound++;
                }
        }
        bool fFeeler = false;
        if (nOutbound >= nMaxOutbound) {
            const int64_t now = GetTimeMicros();
            if (now > nNextFeeler) {
                nNextFeeler = PoissonNextSend(now, FEELER_INTERVAL);
                fFeeler = true;
            } else {
                continue;
            }
        }
        const int64_t nANow = GetAdjustedTime();
        CAddress addrConnect;
        for (int nTries = 0; !interruptNet && nTries < 100; nTries++) {
            CAddrInfo a = addrman.Select(fFeeler);
            if (!a.IsValid() || setConnected.count(a.GetGroup()) || IsLocalAddr(a)) break;
            if (IsLimited(a.GetNetwork())) continue; // -onlynet / no proxy for this network
            if ((a.nServices & nRelevantServices) != nRelevantServices) continue;
            if (nANow - a.nLastTry < 600 && nTries < 30) continue;
            if (a.GetPort() != Params().GetDefaultPort() && nTries < 50) continue;
            addrConnect = a;
            break;
        }
        if (addrConnect.IsValid()) {
            if (fFeeler) {
                // jitter before a feeler connection
                if (!InterruptibleSleep(GetRand(5000))) return;
                LogPrint(BCLog::NET, "Making feeler connection to %s\n", addrConnect.ToString().c_str());
            }
            OpenNetworkConnection(addrConnect, (int)setConnected.size() >= std::min(nMaxConnections - 1, 2), nullptr,
                                  false, fFeeler);
        }
    }
}

std::vector<AddedNodeInfo> CConnman::GetAddedNodeInfo() {
    std::vector<AddedNodeInfo> ret;
    std::vector<std::string> added;
    {
        std::lock_guard<Mutex> l(cs_vAddedNodes);
        added = vAddedNodes;
    }
    std::map<CService, bool> mapConnected;
    std::map<std::string, std::pair<bool, CService>> mapConnectedByName;
    {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        for (CNode* p : vNodes) {
            if (p->addr.IsValid()) mapConnected[p->addr] = p->fInbound;
            if (!p->addrName.empty()) mapConnectedByName[p->addrName] = {p->fInbound, p->addr};
        }
    }
    for (const std::string& s : added) {
        CService svc = LookupNumeric(s, Params().GetDefaultPort());
        AddedNodeInfo info{s, CService(), false, false};
        if (svc.IsValid()) {
            info.resolvedAddress = svc;
            auto it = mapConnected.find(svc);
            if (it != mapConnected.end()) {
                info.fConnected = true;
                info.fInbound = it->second;
            }
        } else {
            auto it = mapConnectedByName.find(s);
            if (it != mapConnectedByName.end()) {
                info.fConnected = true;
                info.fInbound = it->second.first;
                info.resolvedAddress = it->second.second;
            }
        }
        ret.push_back(info);
    }
    return ret;
}

void CConnman::ThreadOpenAddedConnections() {
    {
        std::lock_guard<Mutex> l(cs_vAddedNodes);
        for (const std::string& s : gArgs.GetArgs("-addnode")) vAddedNodes.push_back(s);
    }
    while (!interruptNet) {
        std::vector<AddedNodeInfo> info = GetAddedNodeInfo();
        bool tried = false;
        for (const AddedNodeInfo& i : info) {
            if (!i.fConnected) {
                if (!fNetworkActive) break;
                tried = true;
                CAddress addr(CService(), NODE_NONE);
                OpenNetworkConnection(addr, false, i.strAddedNode.c_str(), false, false, true);
                if (!InterruptibleSleep(500)) return;
            }
        }
        if (!InterruptibleSleep(tried ? 60000 : 2000)) return;
    }
}

std::vector<CAddress> ConvertSeed6(const std::vector<SeedSpec6>& seeds) {
    // fixed seeds look a week or two old, so addrman prefers any fresher address it learns
    static const int64_t nOneWeek = 7 * 24 * 60 * 60;
    std::vector<CAddress> out;
    out.reserve(seeds.size());
    FastRandomContext rng;
    for (const SeedSpec6& s : seeds) {
        CNetAddr ip;
        ip.SetRaw(s.addr);
        CAddress a(CService(ip, s.port), NODE_NETWORK);
        a.nTime = (uint32_t)(GetTime() - (int64_t)rng.randrange(nOneWeek) - nOneWeek);
        out.push_back(a);
    }
    return out;
}

void CConnman::ThreadDNSAddressSeed() {
    // only query DNS seeds when the address book is thin, unless -forcednsseed (reference
    // net.cpp:1582-1660)
    if (!InterruptibleSleep(11000)) return;
    if (addrman.size() > 0 && !fForceDNSSeed) {
        std::lock_guard<CCriticalSection> l(cs_vNodes);
        int n = 0;
        for (CNode* p : vNodes) n += (p->fSuccessfullyConnected && !p->fOneShot && !p->fFeeler && !p->fInbound);
        if (n >= 2) return;
    }
    int found = 0;
    for (const CDNSSeedData& seed : Params().DNSSeeds()) {
        if (interruptNet) return;
        std::vector<CNetAddr> ips;
        if (LookupHost(seed.host, ips, 256, true)) {
            std::vector<CAddress> addrs;
            for (const CNetAddr& ip : ips) {
                CAddress a(CService(ip, (uint16_t)Params().GetDefaultPort()), NODE_NETWORK);
                a.nTime = (uint32_t)(GetTime() - 3 * 24 * 3600 - GetRand(4 * 24 * 3600));
                addrs.push_back(a);
                found++;
            }
            CNetAddr src;
            LookupHost(seed.name, src, true);
            addrman.Add(addrs, src);
        }
    }
    LogPrintf("%d addresses found from DNS seeds\n", found);
}

bool CConnman::ForNode(NodeId id, std::function<bool(CNode*)> func) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (p->GetId() == id) return !p->fDisconnect && func(p);
    return false;
}

void CConnman::ForEachNode(std::function<void(CNode*)> func) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (p->fSuccessfullyConnected && !p->fDisconnect) func(p);
}

void CConnman::Ban(const CNetAddr& addr, BanReason reason, int64_t bantime, bool sinceUnixEpoch) {
    Ban(CSubNet(addr), reason, bantime, sinceUnixEpoch);
}

void CConnman::Ban(const CSubNet& sub, BanReason reason, int64_t bantime, bool sinceUnixEpoch) {
    banman.Ban(sub, reason, bantime, sinceUnixEpoch);
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (sub.Match(p->addr)) p->fDisconnect = true;
    uiInterface.BannedListChanged();
    if (reason == BanReasonManuallyAdded) DumpData();
}

bool CConnman::Unban(const CNetAddr& addr) { return Unban(CSubNet(addr)); }
bool CConnman::Unban(const CSubNet& sub) {
    if (!banman.Unban(sub)) return false;
    uiInterface.BannedListChanged();
    DumpData();
    return true;
}
void CConnman::ClearBanned() {
    banman.ClearBanned();
    uiInterface.BannedListChanged();
    DumpData();
}

bool CConnman::AddNode(const std::string& node) {
    std::lock_guard<Mutex> l(cs_vAddedNodes);
    for (const std::string& s : vAddedNodes)
        if (s == node) return false;
    vAddedNodes.push_back(node);
    return true;
}

bool CConnman::RemoveAddedNode(const std::string& node) {
    std::lock_guard<Mutex> l(cs_vAddedNodes);
    for (auto it = vAddedNodes.begin(); it != vAddedNodes.end(); ++it)
        if (*it == node) {
            vAddedNodes.erase(it);
            return true;
        }
    return false;
}

size_t CConnman::GetNodeCount(NumConnections flags) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    if (flags == CONNECTIONS_ALL) return vNodes.size();
    size_t n = 0;
    for (CNode* p : vNodes)
        if (flags & (p->fInbound ? CONNECTIONS_IN : CONNECTIONS_OUT)) n++;
    return n;
}

void CConnman::GetNodeStats(std::vector<CNodeStats>& v) {
    v.clear();
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes) {
        v.emplace_back();
        p->CopyStats(v.back());
    }
}

bool CConnman::DisconnectNode(const std::string& node) {
    if (CNode* p = FindNode(node)) {
        p->fDisconnect = true;
        return true;
    }
    CService svc = LookupNumeric(node, Params().GetDefaultPort());
    if (svc.IsValid()) {
        if (CNode* p = FindNode(svc)) {
            p->fDisconnect = true;
            return true;
        }
    }
    return false;
}

bool CConnman::DisconnectNode(const CNetAddr& addr) {
    if (CNode* p = FindNode(addr)) {
        p->fDisconnect = true;
        return true;
    }
    return false;
}

bool CConnman::DisconnectNode(NodeId id) {
    std::lock_guard<CCriticalSection> l(cs_vNodes);
    for (CNode* p : vNodes)
        if (p->GetId() == id) {
            p->fDisconnect = true;
            return true;
        }
    return false;
}

int64_t CConnman::PoissonNextSendInbound(int64_t now, int average_interval_seconds) {
    if (nNextInvSendInbound < now) nNextInvSendInbound = PoissonNextSend(now, average_interval_seconds);
    return nNextInvSendInbound;
}

void CConnman::RelayTransaction(const CTransaction& tx) {
    const CInv inv(MSG_TX, tx.GetHash());
    ForEachNode([&](CNode* p) { p->PushInventory(inv); });
}

} // namespace bcp
