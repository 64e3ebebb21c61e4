// Network RPCs.
// Parity: reference src/rpc/net.cpp:747 command table: getconnectioncount, ping,
// getpeerinfo, addnode, disconnectnode, getaddednodeinfo, getnettotals,
// getnetworkinfo, setban, listbanned, clearbanned, setnetworkactive.
#include "net/net.h"
#include "net/net_processing.h"
#include "node/node.h"
#include "node/policy.h"
#include "rpc/server.h"
#include "net/netbase.h"
#include "util/strencodings.h"

namespace bcp {

static CConnman& Connman() {
    CConnman* c = GetConnman();
    if (!c) ThrowRPC(RPC_CLIENT_P2P_DISABLED, "Error: Peer-to-peer functionality missing or disabled");
    return *c;
}

static UniValue getconnectioncount(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getconnectioncount");
    return (int64_t)Connman().GetNodeCount(CONNECTIONS_ALL);
}

static UniValue ping(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "ping");
    Connman().ForEachNode([](CNode* p) { p->fPingQueued = true; });
    Connman().WakeMessageHandler();
    return UniValue::NullUniValue;
}

static UniValue getpeerinfo(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getpeerinfo");
    std::vector<CNodeStats> stats;
    Connman().GetNodeStats(stats);
    UniValue ret(UniValue::VARR);
    for (const CNodeStats& s : stats) {
        UniValue obj(UniValue::VOBJ);
        CNodeStateStats st;
        const bool fState = GetPeerLogic() && GetPeerLogic()->GetNodeStateStats(s.nodeid, st);
        obj.pushKV("id", (int64_t)s.nodeid);
        obj.pushKV("addr", s.addrName);
        if (!s.addrLocal.empty()) obj.pushKV("addrlocal", s.addrLocal);
        obj.pushKV("services", strprintf("%016llx", (unsigned long long)s.nServices));
        obj.pushKV("relaytxes", s.fRelayTxes);
        obj.pushKV("lastsend", s.nLastSend);
        obj.pushKV("lastrecv", s.nLastRecv);
        obj.pushKV("bytessent", (int64_t)s.nSendBytes);
        obj.pushKV("bytesrecv", (int64_t)s.nRecvBytes);
        obj.pushKV("conntime", s.nTimeConnected);
        obj.pushKV("timeoffset", s.nTimeOffset);
        if (s.dPingTime > 0.0) obj.pushKV("pingtime", s.dPingTime);
        if (s.dMinPing > 0.0) obj.pushKV("minping", s.dMinPing);
        if (s.dPingWait > 0.0) obj.pushKV("pingwait", s.dPingWait);
        obj.pushKV("version", s.nVersion);
        obj.pushKV("subver", s.cleanSubVer);
        obj.pushKV("inbound", s.fInbound);
        obj.pushKV("addnode", s.fAddnode);
        obj.pushKV("startingheight", s.nStartingHeight);
        if (fState) {
            obj.pushKV("banscore", st.nMisbehavior);
            obj.pushKV("synced_headers", st.nSyncHeight);
            obj.pushKV("synced_blocks", st.nCommonHeight);
            UniValue heights(UniValue::VARR);
            for (int h : st.vHeightInFlight) heights.push_back(h);
            obj.pushKV("inflight", heights);
        }
        obj.pushKV("whitelisted", s.fWhitelisted);
        UniValue sendPer(UniValue::VOBJ), recvPer(UniValue::VOBJ);
        for (const auto& kv : s.mapSendBytesPerMsgCmd)
            if (kv.second) sendPer.pushKV(kv.first, (int64_t)kv.second);
        for (const auto& kv : s.mapRecvBytesPerMsgCmd)
            if (kv.second) recvPer.pushKV(kv.first, (int64_t)kv.second);
        obj.pushKV("bytessent_per_msg", sendPer);
        obj.pushKV("bytesrecv_per_msg", recvPer);
        ret.push_back(obj);
    }
    return ret;
}

static UniValue addnode(const JSONRPCRequest& req) {
    std::string strCommand;
    if (req.params.size() == 2) strCommand = req.params[1].get_str();
    if (req.params.size() != 2 || (strCommand != "onetry" && strCommand != "add" && strCommand != "remove"))
        ThrowRPC(RPC_INVALID_PARAMS, "addnode \"node\" \"add|remove|onetry\"");
    const std::string node = req.params[0].get_str();
    CConnman& c = Connman();
    if (strCommand == "onetry") {
        CAddress addr;
        c.OpenNetworkConnection(addr, false, node.c_str());
        return UniValue::NullUniValue;
    }
    if (strCommand == "add") {
        if (!c.AddNode(node)) ThrowRPC(RPC_CLIENT_NODE_ALREADY_ADDED, "Error: Node already added");
    } else if (!c.RemoveAddedNode(node)) {
        ThrowRPC(RPC_CLIENT_NODE_NOT_ADDED, "Error: Node has not been added.");
    }
    return UniValue::NullUniValue;
}

// By address, or by node id with an empty/null address (reference net.cpp disconnectnode).
static UniValue disconnectnode(const JSONRPCRequest& req) {
    if (req.params.size() == 0 || req.params.size() > 2)
        ThrowRPC(RPC_INVALID_PARAMS, "disconnectnode \"[address]\" [nodeid]");
    const UniValue& address = req.params[0];
    const UniValue& id = req.params.size() < 2 ? UniValue::NullUniValue : req.params[1];
    bool success;
    if (!address.isNull() && id.isNull()) {
        success = Connman().DisconnectNode(address.get_str());
    } else if (!id.isNull() && (address.isNull() || (address.isStr() && address.get_str().empty()))) {
        success = Connman().DisconnectNode((NodeId)id.get_int64());
    } else {
        ThrowRPC(RPC_INVALID_PARAMS, "Only one of address and nodeid should be provided.");
    }
    if (!success) ThrowRPC(RPC_CLIENT_NODE_NOT_CONNECTED, "Node not found in connected nodes");
    return UniValue::NullUniValue;
}

static UniValue getaddednodeinfo(const JSONRPCRequest& req) {
    if (req.params.size() > 1) ThrowRPC(RPC_INVALID_PARAMS, "getaddednodeinfo ( \"node\" )");
    std::vector<AddedNodeInfo> info = Connman().GetAddedNodeInfo();
    if (req.params.size() == 1 && !req.params[0].isNull()) {
        const std::string want = req.params[0].get_str();
        std::vector<AddedNodeInfo> f;
        for (const AddedNodeInfo& i : info)
            if (i.strAddedNode == want) f.push_back(i);
        if (f.empty()) ThrowRPC(RPC_CLIENT_NODE_NOT_ADDED, "Error: Node has not been added.");
        info = f;
    }
    UniValue ret(UniValue::VARR);
    for (const AddedNodeInfo& i : info) {
        UniValue obj(UniValue::VOBJ);
        obj.pushKV("addednode", i.strAddedNode);
        obj.pushKV("connected", i.fConnected);
        UniValue addrs(UniValue::VARR);
        if (i.fConnected) {
            UniValue a(UniValue::VOBJ);
            a.pushKV("address", i.resolvedAddress.ToString());
            a.pushKV("connected", i.fInbound ? "inbound" : "outbound");
            addrs.push_back(a);
        }
        obj.pushKV("addresses", addrs);
        ret.push_back(obj);
    }
    return ret;
}

static UniValue getnettotals(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getnettotals");
    CConnman& c = Connman();
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("totalbytesrecv", (int64_t)c.GetTotalBytesRecv());
    obj.pushKV("totalbytessent", (int64_t)c.GetTotalBytesSent());
    obj.pushKV("timemillis", GetTimeMillis());
    UniValue up(UniValue::VOBJ);
    up.pushKV("timeframe", (int64_t)c.GetMaxOutboundTimeframe());
    up.pushKV("target", (int64_t)c.GetMaxOutboundTarget());
    up.pushKV("target_reached", c.OutboundTargetReached(false));
    up.pushKV("serve_historical_blocks", !c.OutboundTargetReached(true));
    up.pushKV("bytes_left_in_cycle", (int64_t)c.GetOutboundTargetBytesLeft());
    up.pushKV("time_left_in_cycle", (int64_t)c.GetMaxOutboundTimeLeftInCycle());
    obj.pushKV("uploadtarget", up);
    return obj;
}

static UniValue getnetworkinfo(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getnetworkinfo");
    CConnman* c = GetConnman();
    NodeContext* node = GetNode();
    const uint64_t maxBlock = node && node->chainstate ? node->chainstate->MaxBlockSize() : DEFAULT_MAX_BLOCK_SIZE;
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("version", CLIENT_VERSION);
    obj.pushKV("subversion", UserAgent(maxBlock));
    obj.pushKV("protocolversion", PROTOCOL_VERSION);
    if (c) obj.pushKV("localservices", strprintf("%016llx", (unsigned long long)c->GetLocalServices()));
    obj.pushKV("localrelay", !gArgs.GetBoolArg("-blocksonly", false));
    obj.pushKV("timeoffset", GetTimeOffset());
    if (c) {
        obj.pushKV("networkactive", c->GetNetworkActive());
        obj.pushKV("connections", (int64_t)c->GetNodeCount(CONNECTIONS_ALL));
    }
    UniValue nets(UniValue::VARR);
    for (Network net : {NET_IPV4, NET_IPV6, NET_TOR}) {
        UniValue o(UniValue::VOBJ);
        proxyType proxy;
        const bool haveProxy = GetProxy(net, proxy);
        o.pushKV("name", GetNetworkName(net));
        o.pushKV("limited", IsLimited(net));
        o.pushKV("reachable", IsReachable(net));
        o.pushKV("proxy", haveProxy ? proxy.proxy.ToStringIPPort() : std::string());
        o.pushKV("proxy_randomize_credentials", haveProxy && proxy.randomize_credentials);
        nets.push_back(o);
    }
    obj.pushKV("networks", nets);
    obj.pushKV("relayfee", ValueFromAmount(minRelayTxFee.GetFeePerK()));
    obj.pushKV("incrementalfee", ValueFromAmount(incrementalRelayFee.GetFeePerK()));
    UniValue locals(UniValue::VARR);
    for (const auto& kv : GetLocalAddresses()) {
        UniValue o(UniValue::VOBJ);
        o.pushKV("address", kv.first.ToString());
        o.pushKV("port", kv.second.first);
        o.pushKV("score", kv.second.second);
        locals.push_back(o);
    }
    obj.pushKV("localaddresses", locals);
    obj.pushKV("warnings", node && node->chainstate ? node->chainstate->Warnings() : "");
    return obj;
}

static UniValue setban(const JSONRPCRequest& req) {
    std::string strCommand;
    if (req.params.size() >= 2) strCommand = req.params[1].get_str();
    if (req.params.size() < 2 || (strCommand != "add" && strCommand != "remove"))
        ThrowRPC(RPC_INVALID_PARAMS, "setban \"subnet\" \"add|remove\" (bantime) (absolute)");
    CConnman& c = Connman();
    const std::string s = req.params[0].get_str();
    const bool isSubnet = s.find('/') != std::string::npos;
    CSubNet subNet;
    CNetAddr netAddr;
    if (!isSubnet) {
        if (!LookupHost(s, netAddr, false)) ThrowRPC(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Invalid IP/Subnet");
        subNet = CSubNet(netAddr);
    } else if (!LookupSubNet(s, subNet)) {
        ThrowRPC(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Invalid IP/Subnet");
    }
    if (!subNet.IsValid()) ThrowRPC(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Invalid IP/Subnet");
    if (strCommand == "add") {
        // a single address counts as banned when any banned subnet covers it (reference
        // src/rpc/net.cpp setban: IsBanned(netAddr) for an address, IsBanned(subNet) for a subnet)
        if (isSubnet ? c.IsBanned(subNet) : c.IsBanned(netAddr))
            ThrowRPC(RPC_CLIENT_NODE_ALREADY_ADDED, "Error: IP/Subnet already banned");
        int64_t banTime = 0;
        if (req.params.size() >= 3 && !req.params[2].isNull()) banTime = req.params[2].get_int64();
        bool absolute = false;
        if (req.params.size() == 4 && req.params[3].isTrue()) absolute = true;
        c.Ban(subNet, BanReasonManuallyAdded, banTime, absolute);
    } else if (!c.Unban(subNet)) {
        ThrowRPC(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Unban failed. Requested address/subnet was not previously banned.");
    }
    return UniValue::NullUniValue;
}

static UniValue listbanned(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "listbanned");
    banmap_t m;
    Connman().GetBanned(m);
    UniValue ret(UniValue::VARR);
    for (const auto& kv : m) {
        UniValue o(UniValue::VOBJ);
        o.pushKV("address", kv.first.ToString());
        o.pushKV("banned_until", kv.second.nBanUntil);
        o.pushKV("ban_created", kv.second.nCreateTime);
        o.pushKV("ban_reason", kv.second.BanReasonToString());
        ret.push_back(o);
    }
    return ret;
}

static UniValue clearbanned(const JSONRPCRequest& req) {
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "clearbanned");
    Connman().ClearBanned();
    return UniValue::NullUniValue;
}

static UniValue setnetworkactive(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "setnetworkactive true|false");
    Connman().SetNetworkActive(req.params[0].get_bool());
    return Connman().GetNetworkActive();
}

void RegisterNetRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"network", "getconnectioncount", getconnectioncount, true, {}, "getconnectioncount\nReturns the number of connections to other nodes."},
        {"network", "ping", ping, true, {}, "ping\nRequests that a ping be sent to all other nodes, to measure ping time."},
        {"network", "getpeerinfo", getpeerinfo, true, {}, "getpeerinfo\nReturns data about each connected network node as a json array of objects."},
        {"network", "addnode", addnode, true, {"node", "command"}, "addnode \"node\" \"add|remove|onetry\"\nAttempts to add or remove a node from the addnode list."},
        {"network", "disconnectnode", disconnectnode, true, {"address", "nodeid"}, "disconnectnode \"[address]\" [nodeid]\nImmediately disconnects from the specified peer node, by address or (with an empty address) by node id."},
        {"network", "getaddednodeinfo", getaddednodeinfo, true, {"node"}, "getaddednodeinfo ( \"node\" )\nReturns information about the given added node, or all added nodes."},
        {"network", "getnettotals", getnettotals, true, {}, "getnettotals\nReturns information about network traffic."},
        {"network", "getnetworkinfo", getnetworkinfo, true, {}, "getnetworkinfo\nReturns an object containing various state info regarding P2P networking."},
        {"network", "setban", setban, true, {"subnet", "command", "bantime", "absolute"}, "setban \"subnet\" \"add|remove\" (bantime) (absolute)\nAttempts to add or remove an IP/Subnet from the banned list."},
        {"network", "listbanned", listbanned, true, {}, "listbanned\nList all banned IPs/Subnets."},
        {"network", "clearbanned", clearbanned, true, {}, "clearbanned\nClear all banned IPs."},
        {"network", "setnetworkactive", setnetworkactive, true, {"state"}, "setnetworkactive true|false\nDisable/enable all p2p network activity."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
