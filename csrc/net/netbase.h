// Outbound connection policy: SOCKS5 proxies, per-network reachability, name proxy
// (reference src/netbase.{h,cpp} SetProxy/GetProxy/SetNameProxy/IsProxy, Socks5,
// ConnectSocketByName/ConnectThroughProxy; src/net.cpp SetLimited/IsLimited/IsReachable;
// src/init.cpp -proxy/-onion/-proxyrandomize/-onlynet wiring).
//
// -proxy=<ip:port> routes IPv4/IPv6 (and, as the name proxy, hostnames that are then never
// resolved locally) through a SOCKS5 server; -onion=<ip:port> (default: -proxy) routes .onion
// peers; -proxyrandomize sends fresh random username/password credentials per connection so Tor
// isolates every stream on its own circuit; -onlynet=<ipv4|ipv6|onion> restricts outbound
// connections to the listed networks.
#pragma once
#include "net/netaddress.h"

#include <string>

namespace bcp {

struct proxyType {
    CService proxy;
    bool randomize_credentials = false;
    bool IsValid() const { return proxy.IsValid(); }
};

bool SetProxy(Network net, const proxyType& p);
bool GetProxy(Network net, proxyType& out);
bool IsProxy(const CNetAddr& addr);
bool SetNameProxy(const proxyType& p);
bool HaveNameProxy();
bool GetNameProxy(proxyType& out);
void ClearProxies();

void SetLimited(Network net, bool limited = true);
bool IsLimited(Network net);
bool IsReachable(Network net);
bool IsReachable(const CNetAddr& addr);
Network ParseNetwork(const std::string& name); // "ipv4"/"ipv6"/"onion"/"tor"; NET_UNROUTABLE if unknown
std::string GetNetworkName(Network net);

// Blocking connect of a non-blocking socket with a timeout; returns the fd or -1.
int ConnectDirectly(const CService& addr, int timeoutMs);
// Connect to `proxy`, then SOCKS5 CONNECT to host:port (domain-name form, no local DNS).
// On success returns the connected fd (a plain stream to the destination), else -1;
// *outProxyFailed tells a dead proxy apart from a refused destination.
int ConnectThroughProxy(const proxyType& proxy, const std::string& host, uint16_t port, int timeoutMs,
                        bool* outProxyFailed = nullptr);

} // namespace bcp
