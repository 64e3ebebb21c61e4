// P2P connection manager.
// Parity: reference src/net.{h,cpp}: CNode (per-peer socket, recv message assembly
// with header/checksum validation, send queue with optimistic send, ping/inventory/
// addr relay state, byte counters per command), CConnman (listen/bind/whitelist,
// socket thread, message-handler thread, outbound/feeler/addnode/oneshot connection
// threads, DNS seeding, inbound eviction, ban list, addrman persistence every 900 s,
// nonce-based self-connection detection, network activity toggle, upload target).
//
// Design: a poll(2) socket thread (no select FD_SETSIZE cap) and one message thread
// that round-robins peers, both event-driven by a condition variable.
#pragma once
#include "util/limitedmap.h"
#include "consensus/params.h"
#include "consensus/merkleblock.h"
#include "crypto/hashes.h"
#include "keys/key.h"
#include "net/addrman.h"
#include "net/protocol.h"
#include "primitives/block.h"
#include "util/util.h"

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

// txid -> earliest time (us) any peer may be asked for it; staggers requests for the same
// transaction across peers by 2 minutes each (reference net.cpp mapAlreadyAskedFor).
extern limitedmap<uint256, int64_t> mapAlreadyAskedFor;
extern std::mutex cs_mapAlreadyAskedFor;

typedef int64_t NodeId;
class CConnman;

struct CSerializedNetMsg {
    std::string command;
    std::vector<unsigned char> data;
};

// Builds messages at a peer's negotiated version (reference src/netmessagemaker.h).
class CNetMsgMaker {
public:
    explicit CNetMsgMaker(int version) : nVersion(version) {}
    template <typename... Args> CSerializedNetMsg Make(int flags, const std::string& cmd, const Args&... args) const {
        CSerializedNetMsg m;
        m.command = cmd;
        VectorWriter w(m.data, SER_NETWORK, nVersion | flags);
        int unused[] = {0, (w << args, 0)...};
        (void)unused;
        return m;
    }
    template <typename... Args> CSerializedNetMsg Make(const std::string& cmd, const Args&... args) const {
        return Make(0, cmd, args...);
    }

private:
    int nVersion;
};

struct CNetMessage {
    CMessageHeader hdr;
    std::vector<unsigned char> payload;
    int64_t nTime = 0; // micros received
};

struct CNodeStats {
    NodeId nodeid;
    uint64_t nServices;
    bool fRelayTxes;
    int64_t nLastSend, nLastRecv, nTimeConnected, nTimeOffset;
    std::string addrName;
    int nVersion;
    std::string cleanSubVer;
    bool fInbound, fAddnode, fWhitelisted;
    int nStartingHeight;
    uint64_t nSendBytes, nRecvBytes;
    std::map<std::string, uint64_t> mapSendBytesPerMsgCmd, mapRecvBytesPerMsgCmd;
    double dPingTime, dPingWait, dMinPing;
    std::string addrLocal;
    CAddress addr;
};

class CNode {
public:
    CNode(NodeId id, uint64_t localServices, int startingHeight, int fd, const CAddress& addr, uint64_t keyedNetGroup,
          uint64_t localHostNonce, const std::string& addrName, bool fInbound);
    ~CNode();
    CNode(const CNode&) = delete;

    NodeId GetId() const { return id; }
    uint64_t GetLocalNonce() const { return nLocalHostNonce; }
    uint64_t GetLocalServices() const { return nLocalServices; }
    int GetMyStartingHeight() const { return nMyStartingHeight; }
    int GetRefCount() const { return nRefCount; }
    CNode* AddRef() { nRefCount++; return this; }
    void Release() { nRefCount--; }

    void SetRecvVersion(int v) { nRecvVersion = v; }
    int GetRecvVersion() const { return nRecvVersion; }
    void SetSendVersion(int v) { nSendVersion = v; }
    int GetSendVersion() const { return nSendVersion; }
    // peers below the BCP protocol version receive 80-byte legacy block headers
    bool IsLegacyBlockHeader(int version) const { return version < BCP_HARD_FORK_VERSION; }
    void SetAddrLocal(const CService& a);
    CService GetAddrLocal() const;

    // Parse raw bytes into messages; false on a framing error (peer is disconnected).
    bool ReceiveMsgBytes(const unsigned char* p, size_t n, const unsigned char* magic, bool& complete);

    void PushAddress(const CAddress& a, FastRandomContext& rng);
    void AddAddressKnown(const CAddress& a);
    void AddInventoryKnown(const CInv& inv);
    void PushInventory(const CInv& inv);
    void PushBlockHash(const uint256& hash);
    void AskFor(const CInv& inv);
    void CopyStats(CNodeStats& st) const;
    std::string GetAddrName() const { return addrName; }
    void CloseSocketDisconnect();

    // ---- immutable identity
    const NodeId id;
    const int64_t nTimeConnected;
    const CAddress addr;
    const std::string addrName;
    const bool fInbound;
    const uint64_t nKeyedNetGroup;
    bool fWhitelisted = false;
    bool fFeeler = false;
    bool fOneShot = false;
    bool fAddnode = false;
    bool fClient = false;

    // ---- socket (owned by the socket thread)
    std::mutex cs_hSocket;
    int hSocket;
    std::mutex cs_vSend;
    std::deque<std::vector<unsigned char>> vSendMsg;
    size_t nSendSize = 0, nSendOffset = 0;
    std::atomic<uint64_t> nSendBytes{0};
    std::mutex cs_vRecv;
    std::atomic<uint64_t> nRecvBytes{0};
    std::mutex cs_vProcessMsg;
    std::list<CNetMessage> vProcessMsg;
    size_t nProcessQueueSize = 0;
    std::atomic<bool> fPauseRecv{false};
    std::atomic<bool> fPauseSend{false};
    std::map<std::string, uint64_t> mapSendBytesPerMsgCmd, mapRecvBytesPerMsgCmd;
    std::atomic<int64_t> nLastSend{0}, nLastRecv{0};
    std::atomic<int64_t> nTimeOffset{0};

    // ---- protocol state
    std::atomic<uint64_t> nServices{NODE_NONE};
    std::atomic<int> nVersion{0};
    std::mutex cs_SubVer;
    std::string strSubVer, cleanSubVer;
    std::atomic<int> nStartingHeight{-1};
    std::atomic<bool> fSuccessfullyConnected{false};
    std::atomic<bool> fDisconnect{false};
    std::atomic<bool> fSentAddr{false};
    bool fRelayTxes = false; // guarded by cs_filter
    std::mutex cs_filter;
    std::unique_ptr<CBloomFilter> pfilter;
    std::atomic<bool> fGetAddr{false};
    std::atomic<int64_t> nLastBlockTime{0};

    // addr relay
    std::vector<CAddress> vAddrToSend;
    CRollingBloomFilter addrKnown;
    std::set<uint256> setKnown;
    int64_t nNextAddrSend = 0, nNextLocalAddrSend = 0;

    // inventory (cs_inventory)
    std::mutex cs_inventory;
    CRollingBloomFilter filterInventoryKnown;
    std::set<uint256> setInventoryTxToSend;
    std::vector<uint256> vInventoryBlockToSend;
    std::vector<uint256> vBlockHashesToAnnounce;
    std::multimap<int64_t, CInv> mapAskFor;
    std::set<uint256> setAskFor; // hashes queued in mapAskFor (one request per hash per peer)
    bool fSendMempool = false;
    int64_t nNextInvSend = 0;
    std::atomic<int64_t> timeLastMempoolReq{0};
    uint256 hashContinue;

    // ping
    std::atomic<uint64_t> nPingNonceSent{0};
    std::atomic<int64_t> nPingUsecStart{0};
    std::atomic<int64_t> nPingUsecTime{0};
    std::atomic<int64_t> nMinPingUsecTime{INT64_MAX};
    std::atomic<bool> fPingQueued{false};

    // feefilter
    std::atomic<int64_t> minFeeFilter{0};
    int64_t lastSentFeeFilter = 0;
    int64_t nextSendTimeFeeFilter = 0;

private:
    const uint64_t nLocalHostNonce;
    const uint64_t nLocalServices;
    const int nMyStartingHeight;
    std::atomic<int> nRefCount{0};
    int nSendVersion = INIT_PROTO_VERSION;
    std::atomic<int> nRecvVersion{INIT_PROTO_VERSION};
    mutable std::mutex cs_addrLocal;
    CService addrLocal;
    // partial message assembly
    bool inHeader = true;
    std::vector<unsigned char> hdrbuf;
    CNetMessage curMsg;
    size_t nDataPos = 0;
    std::vector<CNetMessage> completed;
    friend class CConnman;
};

// Message-processing callbacks implemented by net_processing.
class NetEventsInterface {
public:
    virtual ~NetEventsInterface() {}
    virtual void InitializeNode(CNode* pnode) = 0;
    virtual void FinalizeNode(NodeId id, bool& fUpdateConnectionTime) = 0;
    virtual bool ProcessMessages(CNode* pnode, std::atomic<bool>& interrupt) = 0;
    virtual bool SendMessages(CNode* pnode, std::atomic<bool>& interrupt) = 0;
};

enum NumConnections { CONNECTIONS_NONE = 0, CONNECTIONS_IN = 1, CONNECTIONS_OUT = 2, CONNECTIONS_ALL = 3 };

struct AddedNodeInfo {
    std::string strAddedNode;
    CService resolvedAddress;
    bool fConnected;
    bool fInbound;
};

// Local address advertisement (reference net.cpp mapLocalHost / AddLocal / GetLocal).
enum { LOCAL_NONE, LOCAL_IF, LOCAL_BIND, LOCAL_UPNP, LOCAL_MANUAL, LOCAL_MAX };
bool AddLocal(const CService& addr, int nScore = LOCAL_NONE);
bool RemoveLocal(const CService& addr);
bool IsLocalAddr(const CService& addr);
bool GetLocal(CService& addr, const CNetAddr* paddrPeer = nullptr);
CAddress GetLocalAddress(const CNetAddr* paddrPeer, uint64_t nLocalServices);
std::map<CNetAddr, std::pair<int, int>> GetLocalAddresses(); // addr -> (port, score)
extern std::atomic<bool> fListen;
extern std::atomic<bool> fDiscover;

// The chain's compiled-in fixed seeds as addrman entries (reference net.cpp convertSeed6).
std::vector<CAddress> ConvertSeed6(const std::vector<SeedSpec6>& seeds);

class CConnman {
public:
    struct Options {
        uint64_t nLocalServices = NODE_NETWORK;
        uint64_t nRelevantServices = NODE_NETWORK;
        int nMaxConnections = DEFAULT_MAX_PEER_CONNECTIONS;
        int nMaxOutbound = MAX_OUTBOUND_CONNECTIONS;
        int nMaxAddnode = MAX_ADDNODE_CONNECTIONS;
        int nMaxFeeler = 1;
        int nBestHeight = 0;
        NetEventsInterface* events = nullptr;
        size_t nSendBufferMaxSize = 1000 * 1000 * 5;
        size_t nReceiveFloodSize = 1000 * 1000 * 5;
        uint64_t nMaxOutboundTimeframe = 60 * 60 * 24;
        uint64_t nMaxOutboundLimit = 0;
        std::vector<std::string> vSeedNodes;
        std::vector<std::string> vConnect; // -connect: only these
        bool fConnectOnly = false;
        std::vector<CService> vBinds, vWhiteBinds;
        std::vector<CSubNet> vWhitelistedRange;
        bool fListen = true;
        bool fDefaultBinds = false; // wildcard binds: succeed if any family binds
        bool fDNSSeed = true;
        bool fForceDNSSeed = false; // -forcednsseed: query the seeds even with a full address book
        std::string datadir;
    };

    CConnman(uint64_t seed0, uint64_t seed1);
    ~CConnman();
    bool Start(Scheduler* scheduler, const Options& opts, std::string& err);
    void Stop();
    void Interrupt();

    bool GetNetworkActive() const { return fNetworkActive; }
    void SetNetworkActive(bool active);
    bool OpenNetworkConnection(const CAddress& addrConnect, bool fCountFailure, const char* pszDest = nullptr,
                               bool fOneShot = false, bool fFeeler = false, bool fAddnode = false);
    bool CheckIncomingNonce(uint64_t nonce);

    bool ForNode(NodeId id, std::function<bool(CNode*)> func);
    void ForEachNode(std::function<void(CNode*)> func);
    void PushMessage(CNode* pnode, CSerializedNetMsg&& msg);

    // addrman
    size_t GetAddressCount() const { return addrman.size(); }
    void SetServices(const CService& addr, uint64_t nServices) { addrman.SetServices(addr, nServices); }
    void MarkAddressGood(const CAddress& addr) { addrman.Good(addr); }
    void AddNewAddresses(const std::vector<CAddress>& v, const CAddress& src, int64_t penalty = 0) {
        addrman.Add(v, src, penalty);
    }
    std::vector<CAddress> GetAddresses() { return addrman.GetAddr(); }
    CAddrMan& AddrMan() { return addrman; }

    // bans
    void Ban(const CNetAddr& addr, BanReason reason, int64_t bantime = 0, bool sinceUnixEpoch = false);
    void Ban(const CSubNet& sub, BanReason reason, int64_t bantime = 0, bool sinceUnixEpoch = false);
    bool Unban(const CNetAddr& addr);
    bool Unban(const CSubNet& sub);
    void ClearBanned();
    bool IsBanned(const CNetAddr& addr) { return banman.IsBanned(addr); }
    bool IsBanned(const CSubNet& sub) { return banman.IsBanned(sub); }
    void GetBanned(banmap_t& m) { banman.GetBanned(m); }
    void SetBanned(const banmap_t& m) { banman.SetBanned(m); }

    bool AddNode(const std::string& node);
    bool RemoveAddedNode(const std::string& node);
    std::vector<AddedNodeInfo> GetAddedNodeInfo();
    size_t GetNodeCount(NumConnections flags);
    void GetNodeStats(std::vector<CNodeStats>& v);
    bool DisconnectNode(const std::string& node);
    bool DisconnectNode(NodeId id);
    bool DisconnectNode(const CNetAddr& addr);

    uint64_t GetTotalBytesRecv() const { return nTotalBytesRecv; }
    uint64_t GetTotalBytesSent() const { return nTotalBytesSent; }
    void SetMaxOutboundTarget(uint64_t limit) {
        std::lock_guard<Mutex> l(cs_totalBytesSent);
        nMaxOutboundLimit = limit;
    }
    uint64_t GetMaxOutboundTarget() const {
        std::lock_guard<Mutex> l(cs_totalBytesSent);
        return nMaxOutboundLimit;
    }
    uint64_t GetMaxOutboundTimeframe() const {
        std::lock_guard<Mutex> l(cs_totalBytesSent);
        return nMaxOutboundTimeframe;
    }
    bool OutboundTargetReached(bool historicalBlockServingLimit);
    uint64_t GetOutboundTargetBytesLeft();
    uint64_t GetMaxOutboundTimeLeftInCycle();
    uint64_t GetLocalServices() const { return nLocalServices; }
    void SetBestHeight(int h) { nBestHeight = h; }
    int GetBestHeight() const { return nBestHeight; }
    unsigned GetReceiveFloodSize() const { return (unsigned)nReceiveFloodSize; }
    CSipHasher GetDeterministicRandomizer(uint64_t id) const;
    void WakeMessageHandler();
    int64_t PoissonNextSendInbound(int64_t now, int average_interval_seconds);
    void DumpData();
    int GetListenPort() const { return nListenPort; }
    void RelayTransaction(const CTransaction& tx);

private:
    struct ListenSocket {
        int fd;
        bool whitelisted;
    };
    bool BindListenPort(const CService& bind, std::string& err, bool fWhitelisted);
    void AcceptConnection(const ListenSocket& ls);
    CNode* ConnectNode(CAddress addrConnect, const char* pszDest);
    CNode* FindNode(const CNetAddr& ip);
    CNode* FindNode(const std::string& name);
    CNode* FindNode(const CService& addr);
    bool AttemptToEvictConnection();
    bool IsWhitelistedRange(const CNetAddr& addr);
    void SocketSendData(CNode* pnode);
    void ThreadSocketHandler();
    void ThreadMessageHandler();
    void ThreadOpenConnections();
    void ThreadOpenAddedConnections();
    void ThreadDNSAddressSeed();
    void ProcessOneShot();
    void RecordBytesSent(uint64_t n);
    bool InterruptibleSleep(int64_t millis);

    uint64_t nLocalServices = NODE_NETWORK, nRelevantServices = NODE_NETWORK;
    int nMaxConnections = 0, nMaxOutbound = 0, nMaxAddnode = 0, nMaxFeeler = 0;
    size_t nSendBufferMaxSize = 0, nReceiveFloodSize = 0;
    std::atomic<int> nBestHeight{0};
    NetEventsInterface* events = nullptr;
    std::string datadir;
    int nListenPort = 0;

    std::vector<ListenSocket> vhListenSocket;
    std::atomic<bool> fNetworkActive{true};
    bool fFixedSeedsAdded = false; // ThreadOpenConnections only
    CAddrMan addrman;
    BanMan banman;
    Mutex cs_vOneShots;
    std::deque<std::string> vOneShots GUARDED_BY(cs_vOneShots);
    Mutex cs_vAddedNodes;
    std::vector<std::string> vAddedNodes GUARDED_BY(cs_vAddedNodes);
    std::vector<std::string> vConnect;
    bool fConnectOnly = false;
    bool fDNSSeed = true;
    bool fForceDNSSeed = false;
    std::vector<CSubNet> vWhitelistedRange;
    mutable CCriticalSection cs_vNodes{"cs_vNodes"};
    std::vector<CNode*> vNodes GUARDED_BY(cs_vNodes);
    std::list<CNode*> vNodesDisconnected;
    std::atomic<NodeId> nLastNodeId{0};
    std::atomic<uint64_t> nTotalBytesRecv{0}, nTotalBytesSent{0};
    mutable Mutex cs_totalBytesSent;
    uint64_t nMaxOutboundTotalBytesSentInCycle GUARDED_BY(cs_totalBytesSent) = 0;
    uint64_t nMaxOutboundCycleStartTime GUARDED_BY(cs_totalBytesSent) = 0;
    uint64_t nMaxOutboundLimit GUARDED_BY(cs_totalBytesSent) = 0;
    uint64_t nMaxOutboundTimeframe GUARDED_BY(cs_totalBytesSent) = 0;
    const uint64_t nSeed0, nSeed1;
    int64_t nNextInvSendInbound = 0;

    std::mutex mutexMsgProc;
    std::condition_variable condMsgProc;
    bool fMsgProcWake = false;
    std::atomic<bool> flagInterruptMsgProc{false};
    std::atomic<bool> interruptNet{false};
    std::mutex cs_sleep;
    std::condition_variable cv_sleep;
    std::thread threadSocketHandler, threadMessageHandler, threadOpenConnections, threadOpenAddedConnections,
        threadDNSAddressSeed;
    int wakeupPipe[2] = {-1, -1};
    bool started = false;
};

// Process-wide connection manager (set by StartNetwork).
CConnman* GetConnman();
int64_t PoissonNextSend(int64_t nNow, int average_interval_seconds);

} // namespace bcp
