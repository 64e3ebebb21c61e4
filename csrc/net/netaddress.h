// Network addresses.
// Parity: reference src/netaddress.{h,cpp} (CNetAddr 16-byte IPv6/IPv4-mapped storage,
// IsRFC1918/IsLocal/IsRoutable/GetGroup, CService, CSubNet with netmask matching),
// src/netbase.cpp (LookupHost/Lookup/LookupSubNet via getaddrinfo), and
// src/protocol.h CAddress (services + nTime, serialized with a time field when the
// stream is not a GETHASH and version >= CADDR_TIME_VERSION).
#pragma once
#include "primitives/serialize.h"

#include <netinet/in.h>
#include <sys/socket.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace bcp {

enum Network { NET_UNROUTABLE = 0, NET_IPV4, NET_IPV6, NET_TOR, NET_MAX };

class CNetAddr {
public:
    CNetAddr() { memset(ip, 0, 16); }
    explicit CNetAddr(const struct in_addr& v4);
    explicit CNetAddr(const struct in6_addr& v6);
    void SetIPv4(uint32_t hostOrderAddr);
    void SetRaw(const unsigned char* ip16) { memcpy(ip, ip16, 16); }
    bool SetSpecial(const std::string& s); // .onion -> OnionCat range

    bool IsIPv4() const;
    bool IsIPv6() const { return !IsIPv4() && !IsTor(); }
    bool IsTor() const;
    bool IsRFC1918() const;
    bool IsRFC2544() const;
    bool IsRFC3927() const;
    bool IsRFC6598() const;
    bool IsRFC5737() const;
    bool IsRFC3849() const;
    bool IsRFC3964() const;
    bool IsRFC6052() const;
    bool IsRFC4380() const;
    bool IsRFC4862() const;
    bool IsRFC4193() const;
    bool IsRFC6145() const;
    bool IsRFC4843() const;
    bool IsLocal() const;
    bool IsRoutable() const;
    bool IsValid() const;
    bool IsMulticast() const;
    Network GetNetwork() const;
    std::string ToStringIP() const;
    std::string ToString() const { return ToStringIP(); }
    uint32_t GetIPv4() const; // host order, only when IsIPv4()
    bool GetInAddr(struct in_addr* a) const;
    bool GetIn6Addr(struct in6_addr* a) const;
    // Group used by addrman bucketing and outbound diversity (/16 for IPv4, /32 for IPv6).
    std::vector<unsigned char> GetGroup() const;
    uint64_t GetHash() const;
    unsigned char GetByte(int n) const { return ip[15 - n]; }
    const unsigned char* Raw() const { return ip; }

    friend bool operator==(const CNetAddr& a, const CNetAddr& b) { return memcmp(a.ip, b.ip, 16) == 0; }
    friend bool operator!=(const CNetAddr& a, const CNetAddr& b) { return !(a == b); }
    friend bool operator<(const CNetAddr& a, const CNetAddr& b) { return memcmp(a.ip, b.ip, 16) < 0; }

    template <typename S> void Serialize(S& s) const { s.write((const char*)ip, 16); }
    template <typename S> void Unserialize(S& s) { s.read((char*)ip, 16); }

protected:
    unsigned char ip[16]; // network byte order
};

class CService : public CNetAddr {
public:
    CService() {}
    CService(const CNetAddr& a, uint16_t p) : CNetAddr(a), port(p) {}
    uint16_t GetPort() const { return port; }
    void SetPort(uint16_t p) { port = p; }
    bool GetSockAddr(struct sockaddr* sa, socklen_t* len) const;
    bool SetSockAddr(const struct sockaddr* sa);
    std::string ToStringPort() const { return std::to_string(port); }
    std::string ToStringIPPort() const;
    std::string ToString() const { return ToStringIPPort(); }
    std::vector<unsigned char> GetKey() const;

    friend bool operator==(const CService& a, const CService& b) {
        return (const CNetAddr&)a == (const CNetAddr&)b && a.port == b.port;
    }
    friend bool operator!=(const CService& a, const CService& b) { return !(a == b); }
    friend bool operator<(const CService& a, const CService& b) {
        return (const CNetAddr&)a < (const CNetAddr&)b || ((const CNetAddr&)a == (const CNetAddr&)b && a.port < b.port);
    }

    template <typename S> void Serialize(S& s) const {
        CNetAddr::Serialize(s);
        unsigned char p[2] = {(unsigned char)(port >> 8), (unsigned char)port}; // big-endian
        s.write((const char*)p, 2);
    }
    template <typename S> void Unserialize(S& s) {
        CNetAddr::Unserialize(s);
        unsigned char p[2];
        s.read((char*)p, 2);
        port = (uint16_t)((p[0] << 8) | p[1]);
    }

protected:
    uint16_t port = 0;
};

class CSubNet {
public:
    CSubNet() { memset(netmask, 0, 16); }
    CSubNet(const CNetAddr& addr, int bits);
    explicit CSubNet(const CNetAddr& addr); // single host
    CSubNet(const CNetAddr& addr, const CNetAddr& mask);
    bool Match(const CNetAddr& addr) const;
    bool IsValid() const { return valid; }
    std::string ToString() const;
    const CNetAddr& Network() const { return network; }

    friend bool operator==(const CSubNet& a, const CSubNet& b) {
        return a.valid == b.valid && a.network == b.network && memcmp(a.netmask, b.netmask, 16) == 0;
    }
    friend bool operator<(const CSubNet& a, const CSubNet& b) {
        return a.network < b.network || (a.network == b.network && memcmp(a.netmask, b.netmask, 16) < 0);
    }
    template <typename S> void Serialize(S& s) const {
        network.Serialize(s);
        s.write((const char*)netmask, 16);
        uint8_t v = valid;
        ::bcp::Serialize(s, v);
    }
    template <typename S> void Unserialize(S& s) {
        network.Unserialize(s);
        s.read((char*)netmask, 16);
        uint8_t v;
        ::bcp::Unserialize(s, v);
        valid = v != 0;
    }

private:
    CNetAddr network;
    unsigned char netmask[16];
    bool valid = false;
};

// -dns: allow DNS lookups for -addnode, -seednode and -connect (reference netbase.cpp fNameLookup).
extern bool fNameLookup;
// Name resolution (numeric only when fAllowLookup is false).
bool LookupHost(const std::string& name, std::vector<CNetAddr>& out, unsigned maxSolutions, bool fAllowLookup);
bool LookupHost(const std::string& name, CNetAddr& out, bool fAllowLookup);
bool Lookup(const std::string& name, CService& out, int defaultPort, bool fAllowLookup);
bool Lookup(const std::string& name, std::vector<CService>& out, int defaultPort, bool fAllowLookup,
            unsigned maxSolutions);
CService LookupNumeric(const std::string& name, int defaultPort = 0);
bool LookupSubNet(const std::string& s, CSubNet& out);
void SplitHostPort(const std::string& in, int& portOut, std::string& hostOut);

// Network services advertised in version/addr (reference protocol.h ServiceFlags).
enum ServiceFlags : uint64_t {
    NODE_NONE = 0,
    NODE_NETWORK = (1 << 0),
    NODE_GETUTXO = (1 << 1),
    NODE_BLOOM = (1 << 2),
    NODE_XTHIN = (1 << 4),
};


class CAddress : public CService {
public:
    CAddress() {}
    CAddress(const CService& s, uint64_t services) : CService(s), nServices(services) {}
    uint64_t nServices = NODE_NONE;
    uint32_t nTime = 100000000;
    int64_t nLastTry = 0; // memory only (addrman)

    template <typename S> void Serialize(S& s) const {
        if (s.GetType() & SER_DISK) {
            int32_t v = 0;
            ::bcp::Serialize(s, v);
        }
        if ((s.GetType() & SER_DISK) || (s.GetVersion() >= CADDR_TIME_VERSION && !(s.GetType() & SER_GETHASH)))
            ::bcp::Serialize(s, nTime);
        ::bcp::Serialize(s, nServices);
        CService::Serialize(s);
    }
    template <typename S> void Unserialize(S& s) {
        if (s.GetType() & SER_DISK) {
            int32_t v;
            ::bcp::Unserialize(s, v);
        }
        if ((s.GetType() & SER_DISK) || (s.GetVersion() >= CADDR_TIME_VERSION && !(s.GetType() & SER_GETHASH)))
            ::bcp::Unserialize(s, nTime);
        ::bcp::Unserialize(s, nServices);
        CService::Unserialize(s);
    }
};

} // namespace bcp
