#include "net/netaddress.h"
#include "crypto/hashes.h"
#include "util/strencodings.h"

#include <arpa/inet.h>
#include <netdb.h>

#include <algorithm>

namespace bcp {

static const unsigned char kIPv4Prefix[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
// OnionCat prefix fd87:d87e:eb43::/48 used to carry Tor addresses in the IPv6 space.
static const unsigned char kOnionCat[6] = {0xFD, 0x87, 0xD8, 0x7E, 0xEB, 0x43};

CNetAddr::CNetAddr(const struct in_addr& v4) {
    memcpy(ip, kIPv4Prefix, 12);
    memcpy(ip + 12, &v4, 4);
}
CNetAddr::CNetAddr(const struct in6_addr& v6) { memcpy(ip, &v6, 16); }

void CNetAddr::SetIPv4(uint32_t a) {
    memcpy(ip, kIPv4Prefix, 12);
    ip[12] = a >> 24;
    ip[13] = a >> 16;
    ip[14] = a >> 8;
    ip[15] = a;
}

bool CNetAddr::SetSpecial(const std::string& s) {
    const std::string suffix = ".onion";
    if (s.size() > suffix.size() && s.compare(s.size() - suffix.size(), suffix.size(), suffix) == 0) {
        bool invalid = false;
        std::vector<unsigned char> v = DecodeBase32(s.substr(0, s.size() - suffix.size()), &invalid);
        if (invalid || v.size() != 16 - sizeof(kOnionCat)) return false;
        memcpy(ip, kOnionCat, sizeof(kOnionCat));
        memcpy(ip + sizeof(kOnionCat), v.data(), v.size());
        return true;
    }
    return false;
}

bool CNetAddr::IsIPv4() const { return memcmp(ip, kIPv4Prefix, 12) == 0; }
bool CNetAddr::IsTor() const { return memcmp(ip, kOnionCat, sizeof(kOnionCat)) == 0; }
bool CNetAddr::IsRFC1918() const {
    return IsIPv4() &&
           (GetByte(3) == 10 || (GetByte(3) == 192 && GetByte(2) == 168) ||
            (GetByte(3) == 172 && GetByte(2) >= 16 && GetByte(2) <= 31));
}
bool CNetAddr::IsRFC2544() const { return IsIPv4() && GetByte(3) == 198 && (GetByte(2) == 18 || GetByte(2) == 19); }
bool CNetAddr::IsRFC3927() const { return IsIPv4() && GetByte(3) == 169 && GetByte(2) == 254; }
bool CNetAddr::IsRFC6598() const { return IsIPv4() && GetByte(3) == 100 && GetByte(2) >= 64 && GetByte(2) <= 127; }
bool CNetAddr::IsRFC5737() const {
    return IsIPv4() && ((GetByte(3) == 192 && GetByte(2) == 0 && GetByte(1) == 2) ||
                        (GetByte(3) == 198 && GetByte(2) == 51 && GetByte(1) == 100) ||
                        (GetByte(3) == 203 && GetByte(2) == 0 && GetByte(1) == 113));
}
bool CNetAddr::IsRFC3849() const { return GetByte(15) == 0x20 && GetByte(14) == 0x01 && GetByte(13) == 0x0D && GetByte(12) == 0xB8; }
bool CNetAddr::IsRFC3964() const { return GetByte(15) == 0x20 && GetByte(14) == 0x02; }
bool CNetAddr::IsRFC6052() const {
    static const unsigned char p[12] = {0, 0x64, 0xFF, 0x9B, 0, 0, 0, 0, 0, 0, 0, 0};
    return memcmp(ip, p, 12) == 0;
}
bool CNetAddr::IsRFC4380() const { return GetByte(15) == 0x20 && GetByte(14) == 0x01 && GetByte(13) == 0 && GetByte(12) == 0; }
bool CNetAddr::IsRFC4862() const {
    static const unsigned char p[8] = {0xFE, 0x80, 0, 0, 0, 0, 0, 0};
    return memcmp(ip, p, 8) == 0;
}
bool CNetAddr::IsRFC4193() const { return (GetByte(15) & 0xFE) == 0xFC; }
bool CNetAddr::IsRFC6145() const {
    static const unsigned char p[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF, 0, 0};
    return memcmp(ip, p, 12) == 0;
}
bool CNetAddr::IsRFC4843() const {
    return GetByte(15) == 0x20 && GetByte(14) == 0x01 && GetByte(13) == 0x00 && (GetByte(12) & 0xF0) == 0x10;
}
bool CNetAddr::IsLocal() const {
    if (IsIPv4() && (GetByte(3) == 127 || GetByte(3) == 0)) return true;
    static const unsigned char loop6[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
    return memcmp(ip, loop6, 16) == 0;
}
bool CNetAddr::IsMulticast() const { return (IsIPv4() && (GetByte(3) & 0xF0) == 0xE0) || GetByte(15) == 0xFF; }

bool CNetAddr::IsValid() const {
    // reference netaddress.cpp IsValid: reject unspecified, documentation and
    // "none"/broadcast addresses, and the pchIPv4 bug-compat prefix of old versions.
    static const unsigned char oldIPv4[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
    if (memcmp(ip, oldIPv4 + 3, 9) == 0) return false;
    static const unsigned char none6[16] = {};
    if (memcmp(ip, none6, 16) == 0) return false;
    if (IsRFC3849()) return false;
    if (IsIPv4()) {
        const uint32_t a = GetIPv4();
        if (a == 0xFFFFFFFFu || a == 0) return false;
    }
    return true;
}

bool CNetAddr::IsRoutable() const {
    return IsValid() && !(IsRFC1918() || IsRFC2544() || IsRFC3927() || IsRFC4862() || IsRFC6598() || IsRFC5737() ||
                          (IsRFC4193() && !IsTor()) || IsRFC4843() || IsLocal());
}

Network CNetAddr::GetNetwork() const {
    if (!IsRoutable()) return NET_UNROUTABLE;
    if (IsIPv4()) return NET_IPV4;
    if (IsTor()) return NET_TOR;
    return NET_IPV6;
}

uint32_t CNetAddr::GetIPv4() const {
    return ((uint32_t)ip[12] << 24) | ((uint32_t)ip[13] << 16) | ((uint32_t)ip[14] << 8) | ip[15];
}

bool CNetAddr::GetInAddr(struct in_addr* a) const {
    if (!IsIPv4()) return false;
    memcpy(a, ip + 12, 4);
    return true;
}
bool CNetAddr::GetIn6Addr(struct in6_addr* a) const {
    memcpy(a, ip, 16);
    return true;
}

std::string CNetAddr::ToStringIP() const {
    if (IsTor()) return EncodeBase32(ip + 6, 10) + ".onion";
    char buf[INET6_ADDRSTRLEN] = {};
    if (IsIPv4()) {
        struct in_addr a;
        GetInAddr(&a);
        inet_ntop(AF_INET, &a, buf, sizeof(buf));
    } else {
        struct in6_addr a;
        GetIn6Addr(&a);
        inet_ntop(AF_INET6, &a, buf, sizeof(buf));
    }
    return buf;
}

std::vector<unsigned char> CNetAddr::GetGroup() const {
    std::vector<unsigned char> g;
    int nClass = NET_IPV6, nStartByte = 0, nBits = 16;
    if (IsLocal()) {
        nClass = 255;
        nBits = 0;
    }
    if (!IsRoutable()) { // local addresses are unroutable too: one group for all of them
        nClass = NET_UNROUTABLE;
        nBits = 0;
    } else if (IsIPv4() || IsRFC6145() || IsRFC6052()) {
        nClass = NET_IPV4;
        nStartByte = 12;
    } else if (IsRFC3964()) {
        nClass = NET_IPV4;
        nStartByte = 2;
    } else if (IsRFC4380()) {
        g.push_back(NET_IPV4);
        g.push_back(GetByte(3) ^ 0xFF);
        g.push_back(GetByte(2) ^ 0xFF);
        return g;
    } else if (IsTor()) {
        nClass = NET_TOR;
        nStartByte = 6;
        nBits = 4;
    } else if (GetByte(15) == 0x20 && GetByte(14) == 0x01 && GetByte(13) == 0x04 && GetByte(12) == 0x70) {
        nBits = 36; // he.net tunnels
    } else {
        nBits = 32;
    }
    g.push_back((unsigned char)nClass);
    while (nBits >= 8) {
        g.push_back(ip[nStartByte++]);
        nBits -= 8;
    }
    if (nBits > 0) g.push_back(ip[nStartByte] | ((1 << (8 - nBits)) - 1));
    return g;
}

uint64_t CNetAddr::GetHash() const {
    unsigned char h[32];
    Sha256d(ip, 16, h);
    uint64_t r;
    memcpy(&r, h, 8);
    return r;
}

bool CService::GetSockAddr(struct sockaddr* sa, socklen_t* len) const {
    if (IsIPv4()) {
        if (*len < (socklen_t)sizeof(struct sockaddr_in)) return false;
        *len = sizeof(struct sockaddr_in);
        struct sockaddr_in* s4 = (struct sockaddr_in*)sa;
        memset(s4, 0, sizeof(*s4));
        GetInAddr(&s4->sin_addr);
        s4->sin_family = AF_INET;
        s4->sin_port = htons(port);
        return true;
    }
    if (*len < (socklen_t)sizeof(struct sockaddr_in6)) return false;
    *len = sizeof(struct sockaddr_in6);
    struct sockaddr_in6* s6 = (struct sockaddr_in6*)sa;
    memset(s6, 0, sizeof(*s6));
    GetIn6Addr(&s6->sin6_addr);
    s6->sin6_family = AF_INET6;
    s6->sin6_port = htons(port);
    return true;
}

bool CService::SetSockAddr(const struct sockaddr* sa) {
    if (sa->sa_family == AF_INET) {
        const struct sockaddr_in* s4 = (const struct sockaddr_in*)sa;
        *this = CService(CNetAddr(s4->sin_addr), ntohs(s4->sin_port));
        return true;
    }
    if (sa->sa_family == AF_INET6) {
        const struct sockaddr_in6* s6 = (const struct sockaddr_in6*)sa;
        *this = CService(CNetAddr(s6->sin6_addr), ntohs(s6->sin6_port));
        return true;
    }
    return false;
}

std::string CService::ToStringIPPort() const {
    if (IsIPv4() || IsTor()) return ToStringIP() + ":" + ToStringPort();
    return "[" + ToStringIP() + "]:" + ToStringPort();
}

std::vector<unsigned char> CService::GetKey() const {
    std::vector<unsigned char> k(ip, ip + 16);
    k.push_back(port >> 8);
    k.push_back(port & 0xFF);
    return k;
}

CSubNet::CSubNet(const CNetAddr& addr, int bits) : network(addr), valid(true) {
    const int astart = addr.IsIPv4() ? 96 : 0;
    if (bits < 0 || bits > 128 - astart) {
        valid = false;
        return;
    }
    bits += astart;
    memset(netmask, 0, 16);
    // prefix 0xff bytes
    for (int i = 0; i < 16; i++) {
        const int b = std::min(8, std::max(0, bits - 8 * i));
        netmask[i] = (unsigned char)(0xFF00 >> b);
    }
    unsigned char raw[16];
    for (int i = 0; i < 16; i++) raw[i] = addr.Raw()[i] & netmask[i];
    network.SetRaw(raw);
}

CSubNet::CSubNet(const CNetAddr& addr) : network(addr), valid(addr.IsValid()) { memset(netmask, 0xFF, 16); }

// Any mask, contiguous or not (reference netaddress.cpp CSubNet(addr, mask)); an IPv4 mask
// applies to the IPv4 part only.
CSubNet::CSubNet(const CNetAddr& addr, const CNetAddr& mask) : network(addr), valid(true) {
    if (addr.IsIPv4() != mask.IsIPv4()) {
        valid = false;
        return;
    }
    memset(netmask, 0xFF, 16);
    const int start = addr.IsIPv4() ? 12 : 0;
    for (int i = start; i < 16; i++) netmask[i] = mask.Raw()[i];
    unsigned char raw[16];
    for (int i = 0; i < 16; i++) raw[i] = addr.Raw()[i] & netmask[i];
    network.SetRaw(raw);
}

bool CSubNet::Match(const CNetAddr& addr) const {
    if (!valid || !addr.IsValid()) return false;
    for (int i = 0; i < 16; i++)
        if ((addr.Raw()[i] & netmask[i]) != network.Raw()[i]) return false;
    return true;
}

std::string CSubNet::ToString() const {
    int bits = 0;
    bool valid_cidr = true;
    const int start = network.IsIPv4() ? 12 : 0;
    for (int i = start; i < 16; i++) {
        unsigned char m = netmask[i];
        int b = 0;
        while (m & 0x80) {
            b++;
            m <<= 1;
        }
        if (m) valid_cidr = false;
        bits += b;
        if (b < 8 && i + 1 < 16 && netmask[i + 1]) valid_cidr = false;
    }
    if (!valid_cidr) { // the mask itself, printed as an address of the subnet's family
        CNetAddr m;
        unsigned char raw[16];
        memcpy(raw, netmask, 16);
        if (network.IsIPv4()) {
            static const unsigned char mapped[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
            memcpy(raw, mapped, 12);
        }
        m.SetRaw(raw);
        return network.ToString() + "/" + m.ToStringIP();
    }
    return network.ToString() + "/" + std::to_string(bits);
}

void SplitHostPort(const std::string& in, int& portOut, std::string& hostOut) {
    const size_t colon = in.find_last_of(':');
    const bool fHaveColon = colon != std::string::npos;
    const bool fBracketed = fHaveColon && in[0] == '[' && in[colon - 1] == ']';
    const bool fMultiColon = fHaveColon && in.find_last_of(':', colon - 1) != std::string::npos;
    if (fHaveColon && (colon == 0 || fBracketed || !fMultiColon)) {
        char* end = nullptr;
        const long n = strtol(in.c_str() + colon + 1, &end, 10);
        if (end && *end == 0 && n > 0 && n < 0x10000) {
            hostOut = in.substr(0, colon);
            portOut = (int)n;
        } else {
            hostOut = in;
        }
    } else {
        hostOut = in;
    }
    if (hostOut.size() > 0 && hostOut[0] == '[' && hostOut.back() == ']') hostOut = hostOut.substr(1, hostOut.size() - 2);
}

bool fNameLookup = true;

bool LookupHost(const std::string& name, std::vector<CNetAddr>& out, unsigned maxSolutions, bool fAllowLookup) {
    std::string host = name;
    if (host.empty()) return false;
    if (host.size() > 1 && host[0] == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
    CNetAddr special;
    if (special.SetSpecial(host)) {
        out.push_back(special);
        return true;
    }
    struct addrinfo hints;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = fAllowLookup ? AI_ADDRCONFIG : AI_NUMERICHOST;
    struct addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0) return false;
    for (struct addrinfo* ai = res; ai && (maxSolutions == 0 || out.size() < maxSolutions); ai = ai->ai_next) {
        CService s;
        if (s.SetSockAddr(ai->ai_addr)) out.push_back((CNetAddr)s);
    }
    freeaddrinfo(res);
    return !out.empty();
}

bool LookupHost(const std::string& name, CNetAddr& out, bool fAllowLookup) {
    std::vector<CNetAddr> v;
    if (!LookupHost(name, v, 1, fAllowLookup)) return false;
    out = v[0];
    return true;
}

bool Lookup(const std::string& name, std::vector<CService>& out, int defaultPort, bool fAllowLookup,
            unsigned maxSolutions) {
    if (name.empty()) return false;
    int port = defaultPort;
    std::string host;
    SplitHostPort(name, port, host);
    std::vector<CNetAddr> ips;
    if (!LookupHost(host, ips, maxSolutions, fAllowLookup)) return false;
    for (const CNetAddr& a : ips) out.push_back(CService(a, (uint16_t)port));
    return true;
}

bool Lookup(const std::string& name, CService& out, int defaultPort, bool fAllowLookup) {
    std::vector<CService> v;
    if (!Lookup(name, v, defaultPort, fAllowLookup, 1)) return false;
    out = v[0];
    return true;
}

CService LookupNumeric(const std::string& name, int defaultPort) {
    CService s;
    if (!Lookup(name, s, defaultPort, false)) return CService();
    return s;
}

bool LookupSubNet(const std::string& str, CSubNet& out) {
    const size_t slash = str.find_last_of('/');
    CNetAddr network;
    if (!LookupHost(str.substr(0, slash), network, false)) return false;
    if (slash == std::string::npos) {
        out = CSubNet(network);
        return out.IsValid();
    }
    const std::string rest = str.substr(slash + 1);
    char* end = nullptr;
    const long n = strtol(rest.c_str(), &end, 10);
    if (end && *end == 0 && !rest.empty()) {
        out = CSubNet(network, (int)n);
        return out.IsValid();
    }
    // a netmask written as an address
    CNetAddr mask;
    if (!LookupHost(rest, mask, false)) return false;
    out = CSubNet(network, mask);
    return out.IsValid();
}

} // namespace bcp
