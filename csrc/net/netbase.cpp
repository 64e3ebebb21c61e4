// SOCKS5 proxying and outbound reachability; see netbase.h.
#include "net/netbase.h"

#include "keys/key.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <fcntl.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <unistd.h>

#include <cerrno>
#include <mutex>

namespace bcp {

namespace {
std::mutex g_cs;
proxyType g_proxies[NET_MAX];
proxyType g_nameProxy;
bool g_limited[NET_MAX] = {};

// SOCKS5 (RFC 1928/1929) constants
enum : uint8_t {
    SOCKS5_VERSION = 0x05,
    METHOD_NOAUTH = 0x00,
    METHOD_USER_PASS = 0x02,
    CMD_CONNECT = 0x01,
    ATYP_DOMAIN = 0x03,
    ATYP_IPV4 = 0x01,
    ATYP_IPV6 = 0x04,
};

// Wait until fd is readable/writable or the deadline passes.
bool WaitFd(int fd, short events, int64_t deadlineMs) {
    while (true) {
        const int64_t left = deadlineMs - GetTimeMillis();
        if (left <= 0) return false;
        struct pollfd p = {fd, events, 0};
        const int rc = poll(&p, 1, (int)std::min<int64_t>(left, 1000));
        if (rc > 0) return true;
        if (rc < 0 && errno != EINTR) return false;
    }
}

bool SendAll(int fd, const std::vector<uint8_t>& buf, int64_t deadlineMs) {
    size_t off = 0;
    while (off < buf.size()) {
        const ssize_t n = send(fd, buf.data() + off, buf.size() - off, MSG_NOSIGNAL);
        if (n > 0) {
            off += (size_t)n;
            continue;
        }
        if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) {
            if (!WaitFd(fd, POLLOUT, deadlineMs)) return false;
            continue;
        }
        return false;
    }
    return true;
}

bool RecvExact(int fd, uint8_t* out, size_t len, int64_t deadlineMs) {
    size_t off = 0;
    while (off < len) {
        const ssize_t n = recv(fd, out + off, len - off, 0);
        if (n > 0) {
            off += (size_t)n;
            continue;
        }
        if (n == 0) return false;
        if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) {
            if (!WaitFd(fd, POLLIN, deadlineMs)) return false;
            continue;
        }
        return false;
    }
    return true;
}

const char* Socks5ErrorString(uint8_t err) {
    switch (err) {
    case 0x01: return "general failure";
    case 0x02: return "connection not allowed";
    case 0x03: return "network unreachable";
    case 0x04: return "host unreachable";
    case 0x05: return "connection refused";
    case 0x06: return "TTL expired";
    case 0x07: return "protocol error";
    case 0x08: return "address type not supported";
    default: return "unknown";
    }
}
} // namespace

bool SetProxy(Network net, const proxyType& p) {
    if (net <= NET_UNROUTABLE || net >= NET_MAX || !p.IsValid()) return false;
    std::lock_guard<std::mutex> l(g_cs);
    g_proxies[net] = p;
    return true;
}
bool GetProxy(Network net, proxyType& out) {
    if (net <= NET_UNROUTABLE || net >= NET_MAX) return false;
    std::lock_guard<std::mutex> l(g_cs);
    if (!g_proxies[net].IsValid()) return false;
    out = g_proxies[net];
    return true;
}
bool IsProxy(const CNetAddr& addr) {
    std::lock_guard<std::mutex> l(g_cs);
    for (int i = 0; i < NET_MAX; ++i)
        if (g_proxies[i].IsValid() && addr == (CNetAddr)g_proxies[i].proxy) return true;
    return false;
}
bool SetNameProxy(const proxyType& p) {
    if (!p.IsValid()) return false;
    std::lock_guard<std::mutex> l(g_cs);
    g_nameProxy = p;
    return true;
}
bool HaveNameProxy() {
    std::lock_guard<std::mutex> l(g_cs);
    return g_nameProxy.IsValid();
}
bool GetNameProxy(proxyType& out) {
    std::lock_guard<std::mutex> l(g_cs);
    if (!g_nameProxy.IsValid()) return false;
    out = g_nameProxy;
    return true;
}
void ClearProxies() {
    std::lock_guard<std::mutex> l(g_cs);
    for (auto& p : g_proxies) p = proxyType();
    g_nameProxy = proxyType();
    for (bool& b : g_limited) b = false;
}

void SetLimited(Network net, bool limited) {
    if (net == NET_UNROUTABLE || net >= NET_MAX) return;
    std::lock_guard<std::mutex> l(g_cs);
    g_limited[net] = limited;
}
bool IsLimited(Network net) {
    if (net >= NET_MAX) return true;
    std::lock_guard<std::mutex> l(g_cs);
    return g_limited[net];
}
bool IsReachable(Network net) { return !IsLimited(net); }
bool IsReachable(const CNetAddr& addr) { return IsReachable(addr.GetNetwork()); }

Network ParseNetwork(const std::string& nameIn) {
    std::string name = nameIn;
    for (char& c : name) c = (char)tolower((unsigned char)c);
    if (name == "ipv4") return NET_IPV4;
    if (name == "ipv6") return NET_IPV6;
    if (name == "onion" || name == "tor") return NET_TOR;
    return NET_UNROUTABLE;
}
std::string GetNetworkName(Network net) {
    switch (net) {
    case NET_IPV4: return "ipv4";
    case NET_IPV6: return "ipv6";
    case NET_TOR: return "onion";
    default: return "";
    }
}

int ConnectDirectly(const CService& addr, int timeoutMs) {
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (!addr.GetSockAddr((struct sockaddr*)&ss, &len)) return -1;
    const int fd = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
    if (fd < 0) return -1;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
    int rc = connect(fd, (struct sockaddr*)&ss, len);
    if (rc != 0 && errno == EINPROGRESS) {
        struct pollfd pfd = {fd, POLLOUT, 0};
        rc = poll(&pfd, 1, timeoutMs);
        int soerr = 0;
        socklen_t sl = sizeof(soerr);
        rc = (rc == 1 && getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) == 0 && soerr == 0) ? 0 : -1;
    }
    if (rc != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

int ConnectThroughProxy(const proxyType& proxy, const std::string& host, uint16_t port, int timeoutMs,
                        bool* outProxyFailed) {
    if (outProxyFailed) *outProxyFailed = true;
    if (host.size() > 255) return -1;
    const int fd = ConnectDirectly(proxy.proxy, timeoutMs);
    if (fd < 0) {
        LogPrintf("Failed to connect to proxy %s\n", proxy.proxy.ToStringIPPort().c_str());
        return -1;
    }
    const int64_t deadline = GetTimeMillis() + timeoutMs;
    auto fail = [&](const char* why) {
        LogPrint(BCLog::PROXY, "SOCKS5 connect to %s:%d failed: %s\n", host.c_str(), port, why);
        close(fd);
        return -1;
    };
    // greeting: offer user/pass auth when randomizing credentials (Tor stream isolation)
    std::vector<uint8_t> greet = {SOCKS5_VERSION, 0x01, METHOD_NOAUTH};
    if (proxy.randomize_credentials) greet = {SOCKS5_VERSION, 0x02, METHOD_NOAUTH, METHOD_USER_PASS};
    if (!SendAll(fd, greet, deadline)) return fail("error sending greeting");
    uint8_t sel[2];
    if (!RecvExact(fd, sel, 2, deadline)) return fail("error reading method selection");
    if (sel[0] != SOCKS5_VERSION) return fail("proxy is not SOCKS5");
    if (sel[1] == METHOD_USER_PASS && proxy.randomize_credentials) {
        unsigned char r[8];
        GetRandBytes(r, sizeof(r));
        const std::string user = HexStr(r, r + 4), pass = HexStr(r + 4, r + 8);
        std::vector<uint8_t> auth = {0x01, (uint8_t)user.size()};
        auth.insert(auth.end(), user.begin(), user.end());
        auth.push_back((uint8_t)pass.size());
        auth.insert(auth.end(), pass.begin(), pass.end());
        if (!SendAll(fd, auth, deadline)) return fail("error sending credentials");
        uint8_t ar[2];
        if (!RecvExact(fd, ar, 2, deadline) || ar[0] != 0x01 || ar[1] != 0x00) return fail("proxy rejected credentials");
    } else if (sel[1] != METHOD_NOAUTH) {
        return fail("proxy requested an unsupported authentication method");
    }
    // CONNECT by domain name: the proxy resolves (no DNS leak for names and .onion)
    std::vector<uint8_t> req = {SOCKS5_VERSION, CMD_CONNECT, 0x00, ATYP_DOMAIN, (uint8_t)host.size()};
    req.insert(req.end(), host.begin(), host.end());
    req.push_back((uint8_t)(port >> 8));
    req.push_back((uint8_t)(port & 0xff));
    if (!SendAll(fd, req, deadline)) return fail("error sending CONNECT");
    uint8_t rep[4];
    if (!RecvExact(fd, rep, 4, deadline)) return fail("error reading CONNECT reply");
    if (rep[0] != SOCKS5_VERSION) return fail("malformed CONNECT reply");
    if (rep[1] != 0x00) {
        if (outProxyFailed) *outProxyFailed = false; // the proxy answered: the destination is at fault
        return fail(Socks5ErrorString(rep[1]));
    }
    size_t skip = 0; // bound address + port
    if (rep[3] == ATYP_IPV4) skip = 4 + 2;
    else if (rep[3] == ATYP_IPV6) skip = 16 + 2;
    else if (rep[3] == ATYP_DOMAIN) {
        uint8_t l;
        if (!RecvExact(fd, &l, 1, deadline)) return fail("error reading bound address");
        skip = l + 2u;
    } else {
        return fail("unknown bound address type");
    }
    uint8_t tmp[300];
    if (!RecvExact(fd, tmp, skip, deadline)) return fail("error reading bound address");
    if (outProxyFailed) *outProxyFailed = false;
    LogPrint(BCLog::PROXY, "SOCKS5 connected %s:%d via %s\n", host.c_str(), port, proxy.proxy.ToStringIPPort().c_str());
    return fd;
}

} // namespace bcp
