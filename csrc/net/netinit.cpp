// Network subsystem start/stop for bcpd (reference src/init.cpp AppInitMain step 6/11:
// -listen/-bind/-whitebind/-whitelist/-connect/-seednode/-addnode/-externalip/
// -maxconnections/-maxuploadtarget/-peerbloomfilters handling and CConnman::Start).
#include "net/net.h"
#include "net/net_processing.h"
#include "net/netbase.h"
#include "node/node.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "util/strencodings.h"

#include <functional>

namespace bcp {

extern std::function<void(const uint256&)> g_relayTransaction;

void StartTorControl(NodeContext& node, int listenPort);
void StartMapPort(int port);
void StopMapPort();
void StopTorControl();

static std::unique_ptr<CConnman> g_connman;
static std::unique_ptr<PeerLogicValidation> g_peerLogic;

std::string NetHelp() {
    std::string s = "\nConnection options:\n";
    const std::pair<const char*, const char*> opts[] = {
        {"-addnode=<ip>", "Add a node to connect to and attempt to keep the connection open"},
        {"-banscore=<n>", "Threshold for disconnecting misbehaving peers (default: 100)"},
        {"-bantime=<n>", "Number of seconds to keep misbehaving peers from reconnecting (default: 86400)"},
        {"-bind=<addr>", "Bind to given address and always listen on it"},
        {"-connect=<ip>", "Connect only to the specified node(s); -connect=0 disables automatic connections"},
        {"-discover", "Discover own IP addresses (default: 1 when listening and no -externalip)"},
        {"-dns", "Allow DNS lookups for -addnode, -seednode and -connect (default: 1)"},
        {"-dnsseed", "Query for peer addresses via DNS lookup, if low on addresses (default: 1 unless -connect)"},
        {"-forcednsseed", "Always query for peer addresses via DNS lookup (default: 0)"},
        {"-maxreceivebuffer=<n>", "Maximum per-connection receive buffer, <n>*1000 bytes (default: 5000)"},
        {"-maxsendbuffer=<n>", "Maximum per-connection send buffer, <n>*1000 bytes (default: 1000)"},
        {"-externalip=<ip>", "Specify your own public address"},
        {"-listen", "Accept connections from outside (default: 1 if no -connect)"},
        {"-maxconnections=<n>", "Maintain at most <n> connections to peers (default: 125)"},
        {"-maxuploadtarget=<n>", "Tries to keep outbound traffic under the given target (in MiB per 24h), 0 = no limit"},
        {"-peerbloomfilters", "Support filtering of blocks and transaction with bloom filters (default: 1)"},
        {"-port=<port>", "Listen for connections on <port> (default: 8337, testnet: 18337, regtest: 18444)"},
        {"-seednode=<ip>", "Connect to a node to retrieve peer addresses, and disconnect"},
        {"-timeout=<n>", "Specify connection timeout in milliseconds (default: 5000)"},
        {"-peertimeout=<n>", "Seconds a new connection has to send its first messages and complete the version handshake (default: 60)"},
        {"-blockreconstructionextratxn=<n>", "Extra transactions to keep in memory for compact block reconstructions (default: 100)"},
        {"-feefilter", "Tell peers the minimum fee rate of transactions to relay to us (default: 1)"},
        {"-uacomment=<cmt>", "Append comment to the user agent string"},
        {"-upnpdiscover=<ip:port>", "SSDP multicast target for UPnP gateway discovery (default: 239.255.255.250:1900)"},
        {"-whitelistrelay", "Accept relayed transactions received from whitelisted peers even when not relaying transactions (default: 1)"},
        {"-whitelistforcerelay", "Force relay of transactions from whitelisted peers even if they violate local relay policy (default: 1)"},
        {"-whitebind=<addr>", "Bind to given address and whitelist peers connecting to it"},
        {"-whitelist=<IP/netmask>", "Whitelist peers connecting from the given IP address or CIDR netmask"},
        {"-blocksonly", "Whether to operate in a blocks only mode (default: 0)"},
        {"-maxorphantx=<n>", "Keep at most <n> unconnectable transactions in memory (default: 100)"},
        {"-listenonion", "Automatically create Tor hidden service (default: 1)"},
        {"-torcontrol=<ip>:<port>", "Tor control port to use if onion listening enabled (default: 127.0.0.1:9051)"},
        {"-torpassword=<pass>", "Tor control port password (default: empty)"},
        {"-proxy=<ip:port>", "Connect through SOCKS5 proxy"},
        {"-onion=<ip:port>", "Use separate SOCKS5 proxy to reach peers via Tor hidden services (default: -proxy)"},
        {"-proxyrandomize", "Randomize credentials for every proxy connection. This enables Tor stream isolation (default: 1)"},
        {"-upnp", "Use UPnP to map the listening port (default: 0)"},
        {"-onlynet=<net>", "Only connect to nodes in network <net> (ipv4, ipv6 or onion)"},
    };
    for (const auto& o : opts) s += strprintf("  %-32s %s\n", o.first, o.second);
    return s;
}

// -onlynet / -proxy / -onion (reference init.cpp AppInitMain step 6)
static bool SetupProxies(std::string& err) {
    ClearProxies();
    const std::vector<std::string> onlynets = gArgs.GetArgs("-onlynet");
    if (!onlynets.empty()) {
        bool allow[NET_MAX] = {};
        for (const std::string& n : onlynets) {
            const Network net = ParseNetwork(n);
            if (net == NET_UNROUTABLE) {
                err = "Unknown network specified in -onlynet: '" + n + "'";
                return false;
            }
            allow[net] = true;
        }
        for (int n = NET_IPV4; n < NET_MAX; ++n) SetLimited((Network)n, !allow[n]);
    }
    const bool randomize = gArgs.GetBoolArg("-proxyrandomize", true);
    const std::string proxyArg = gArgs.GetArg("-proxy", "");
    if (!proxyArg.empty() && proxyArg != "0") {
        CService svc = LookupNumeric(proxyArg, 9050);
        if (!svc.IsValid()) {
            err = "Invalid -proxy address: '" + proxyArg + "'";
            return false;
        }
        proxyType p;
        p.proxy = svc;
        p.randomize_credentials = randomize;
        SetProxy(NET_IPV4, p);
        SetProxy(NET_IPV6, p);
        SetProxy(NET_TOR, p);
        SetNameProxy(p);
    }
    const std::string onionArg = gArgs.GetArg("-onion", "");
    if (onionArg == "0") {
        SetLimited(NET_TOR); // -onion=0: no onion peers at all
    } else if (!onionArg.empty()) {
        CService svc = LookupNumeric(onionArg, 9050);
        if (!svc.IsValid()) {
            err = "Invalid -onion address: '" + onionArg + "'";
            return false;
        }
        proxyType p;
        p.proxy = svc;
        p.randomize_credentials = randomize;
        SetProxy(NET_TOR, p); // reachability of onion peers stays as -onlynet decided
    } else if (proxyArg.empty() || proxyArg == "0") {
        SetLimited(NET_TOR); // no proxy that could reach .onion
    }
    return true;
}

bool StartNetwork(NodeContext& node, std::string& err) {
    const CChainParams& params = *node.params;
    if (!SetupProxies(err)) return false;
    CConnman::Options o;
    std::vector<std::string> connect = gArgs.GetArgs("-connect");
    const bool connectDisabled = connect.size() == 1 && connect[0] == "0";
    if (connectDisabled) connect.clear();
    o.vConnect = connect;
    o.fConnectOnly = gArgs.IsArgSet("-connect");
    const bool listenDefault = !gArgs.IsArgSet("-connect");
    fListen = gArgs.GetBoolArg("-listen", listenDefault);
    o.fListen = fListen;
    fDiscover = gArgs.GetBoolArg("-discover", fListen && !gArgs.IsArgSet("-externalip"));
    o.fDNSSeed = gArgs.GetBoolArg("-dnsseed", !o.fConnectOnly && !gArgs.IsArgSet("-seednode"));
    o.fForceDNSSeed = gArgs.GetBoolArg("-forcednsseed", false);
    o.vSeedNodes = gArgs.GetArgs("-seednode");
    fNameLookup = gArgs.GetBoolArg("-dns", true);
    // per-connection buffers in kB (reference init.cpp:2205-2207)
    o.nSendBufferMaxSize = 1000 * (size_t)std::max<int64_t>(gArgs.GetArg("-maxsendbuffer", (int64_t)1000), 0);
    o.nReceiveFloodSize = 1000 * (size_t)std::max<int64_t>(gArgs.GetArg("-maxreceivebuffer", (int64_t)5000), 0);
    o.nMaxConnections = (int)gArgs.GetArg("-maxconnections", (int64_t)DEFAULT_MAX_PEER_CONNECTIONS);
    o.nLocalServices = NODE_NETWORK;
    if (gArgs.GetBoolArg("-peerbloomfilters", true)) o.nLocalServices |= NODE_BLOOM;
    if (gArgs.GetArg("-prune", (int64_t)0) > 0) o.nLocalServices &= ~(uint64_t)NODE_NETWORK;
    o.nRelevantServices = NODE_NETWORK;
    o.nMaxOutboundLimit = (uint64_t)gArgs.GetArg("-maxuploadtarget", (int64_t)0) * 1024 * 1024;
    o.nBestHeight = node.chainstate->HeightNow();
    o.datadir = node.datadir;
    const int port = (int)gArgs.GetArg("-port", (int64_t)params.GetDefaultPort());
    for (const std::string& b : gArgs.GetArgs("-bind")) {
        CService s;
        if (!Lookup(b, s, port, false)) {
            err = "Cannot resolve -bind address: '" + b + "'";
            return false;
        }
        o.vBinds.push_back(s);
    }
    for (const std::string& b : gArgs.GetArgs("-whitebind")) {
        CService s;
        if (!Lookup(b, s, 0, false) || s.GetPort() == 0) {
            err = "Need to specify a port with -whitebind: '" + b + "'";
            return false;
        }
        o.vWhiteBinds.push_back(s);
    }
    if (o.fListen && o.vBinds.empty() && o.vWhiteBinds.empty()) {
        struct in6_addr any6 = IN6ADDR_ANY_INIT;
        struct in_addr any4;
        any4.s_addr = INADDR_ANY;
        o.vBinds.push_back(CService(CNetAddr(any4), (uint16_t)port));
        o.vBinds.push_back(CService(CNetAddr(any6), (uint16_t)port));
        o.fDefaultBinds = true; // either family may be missing in a container
    }
    for (const std::string& w : gArgs.GetArgs("-whitelist")) {
        CSubNet sub;
        if (!LookupSubNet(w, sub) || !sub.IsValid()) {
            err = "Invalid netmask specified in -whitelist: '" + w + "'";
            return false;
        }
        o.vWhitelistedRange.push_back(sub);
    }
    for (const std::string& e : gArgs.GetArgs("-externalip")) {
        CService s;
        if (Lookup(e, s, port, false)) AddLocal(s, LOCAL_MANUAL);
    }

    g_connman.reset(new CConnman(GetRand(UINT64_MAX), GetRand(UINT64_MAX)));
    g_peerLogic.reset(new PeerLogicValidation(g_connman.get(), node.chainstate.get(), node.mempool.get()));
    o.events = g_peerLogic.get();
    GetMainSignals().Register(g_peerLogic.get());
    node.connman = g_connman.get();
    g_relayTransaction = [&node](const uint256& txid) {
        CTransactionRef tx = node.mempool->get(txid);
        if (tx && g_peerLogic) g_peerLogic->RelayTransaction(*tx);
    };
    if (!g_connman->Start(node.scheduler.get(), o, err)) {
        GetMainSignals().Unregister(g_peerLogic.get());
        node.connman = nullptr;
        g_peerLogic.reset();
        g_connman.reset();
        return false;
    }
    StartTorControl(node, port);
    if (gArgs.GetBoolArg("-upnp", false) && o.fListen) StartMapPort(port);
    LogPrintf("Network started: listen=%d port=%d services=%llx\n", (int)o.fListen, port,
              (unsigned long long)o.nLocalServices);
    return true;
}

void StopNetwork(NodeContext& node) {
    if (!g_connman) return;
    StopMapPort();
    StopTorControl();
    g_relayTransaction = nullptr;
    g_connman->Interrupt();
    g_connman->Stop();
    if (g_peerLogic) GetMainSignals().Unregister(g_peerLogic.get());
    node.connman = nullptr;
    g_peerLogic.reset();
    g_connman.reset();
}

} // namespace bcp
