// Address classification, host:port splitting, numeric lookup, subnets and address groups.
// Parity: reference src/test/netbase_tests.cpp (netbase_networks/properties/splithost/
// lookupnumeric, onioncat_test, subnet_test, netbase_getgroup). The cases here are generated or
// chosen independently: every prefix length and its dotted mask, other members of each RFC range.
#include "net/netaddress.h"
#include "test/unittest.h"
#include "util/strencodings.h"

namespace bcp {
namespace {

CNetAddr IP(const std::string& s) {
    CNetAddr a;
    LookupHost(s, a, false);
    return a;
}
CSubNet Net(const std::string& s) {
    CSubNet n;
    LookupSubNet(s, n);
    return n;
}

std::string DottedMask(int bits) {
    uint32_t m = bits == 0 ? 0 : 0xFFFFFFFFu << (32 - bits);
    return strprintf("%u.%u.%u.%u", m >> 24, (m >> 16) & 255, (m >> 8) & 255, m & 255);
}

} // namespace

TEST_CASE(netbase_tests, networks) {
    CHECK(IP("127.0.0.2").GetNetwork() == NET_UNROUTABLE);
    CHECK(IP("::1").GetNetwork() == NET_UNROUTABLE);
    CHECK(IP("10.20.30.40").GetNetwork() == NET_UNROUTABLE); // private: not routable
    CHECK(IP("93.184.216.34").GetNetwork() == NET_IPV4);
    CHECK(IP("2a00:1450:4001::200e").GetNetwork() == NET_IPV6);
    CHECK(IP("fd87:d87e:eb43:1:2:3:4:5").GetNetwork() == NET_TOR);
}

TEST_CASE(netbase_tests, properties) {
    CHECK(IP("8.8.4.4").IsIPv4());
    CHECK(IP("::ffff:10.1.1.1").IsIPv4()); // mapped
    CHECK(IP("2001:db8::7").IsIPv6());
    for (const char* p : {"10.255.0.1", "172.16.0.1", "172.20.9.9", "192.168.200.3"}) CHECK(IP(p).IsRFC1918());
    for (const char* p : {"172.15.255.255", "172.32.0.0", "11.0.0.1", "192.169.0.1"}) CHECK(!IP(p).IsRFC1918());
    CHECK(IP("2001:db8:1234::").IsRFC3849());
    CHECK(IP("169.254.100.7").IsRFC3927());
    CHECK(IP("2002:c000:0204::1").IsRFC3964());
    CHECK(IP("fc12::1").IsRFC4193());
    CHECK(IP("fdaa::1").IsRFC4193());
    CHECK(IP("2001:0:1::").IsRFC4380());
    CHECK(IP("2001:1f::1").IsRFC4843());
    CHECK(IP("fe80::1:2").IsRFC4862());
    CHECK(IP("64:ff9b::1.2.3.4").IsRFC6052());
    CHECK(IP("198.18.5.5").IsRFC2544());
    CHECK(IP("100.64.1.1").IsRFC6598());
    CHECK(IP("203.0.113.9").IsRFC5737());
    CHECK(IP("127.200.1.1").IsLocal());
    CHECK(IP("::1").IsLocal());
    CHECK(IP("1.1.1.1").IsRoutable());
    CHECK(IP("2a01:4f8::1").IsRoutable());
    CHECK(!IP("192.168.0.1").IsRoutable());
    CHECK(!IP("fe80::1").IsRoutable());
    CHECK(IP("127.0.0.1").IsValid());
    CHECK(!IP("0.0.0.0").IsValid());
    CHECK(!CNetAddr().IsValid());
}

TEST_CASE(netbase_tests, splithost) {
    struct Case {
        const char* in;
        const char* host;
        int port;
    } cases[] = {
        {"example.net", "example.net", -1},       {"[example.net]", "example.net", -1},
        {"example.net:123", "example.net", 123}, {"[example.net]:123", "example.net", 123},
        {"10.1.2.3", "10.1.2.3", -1},             {"10.1.2.3:18444", "10.1.2.3", 18444},
        {"[10.1.2.3]", "10.1.2.3", -1},           {"[10.1.2.3]:18444", "10.1.2.3", 18444},
        {"::ffff:10.1.2.3", "::ffff:10.1.2.3", -1}, {"[::ffff:10.1.2.3]:9", "::ffff:10.1.2.3", 9},
        {"[::]:65535", "::", 65535},              {"::12", "::12", -1},
        {":7", "", 7},                            {"[]:7", "", 7},
        {"", "", -1},
    };
    for (const Case& c : cases) {
        std::string host;
        int port = -1;
        SplitHostPort(c.in, port, host);
        CHECK_EQ(host, std::string(c.host));
        CHECK_EQ(port, c.port);
    }
}

TEST_CASE(netbase_tests, lookupnumeric) {
    auto canon = [](const std::string& s) { return LookupNumeric(s, 4242).ToString(); };
    CHECK_EQ(canon("10.0.0.9"), std::string("10.0.0.9:4242"));
    CHECK_EQ(canon("10.0.0.9:1"), std::string("10.0.0.9:1"));
    CHECK_EQ(canon("::ffff:10.0.0.9"), std::string("10.0.0.9:4242"));
    CHECK_EQ(canon("::"), std::string("[::]:4242"));
    CHECK_EQ(canon("[::]:80"), std::string("[::]:80"));
    CHECK_EQ(canon("[10.0.0.9]"), std::string("10.0.0.9:4242"));
    CHECK_EQ(canon("2001:db8::1"), std::string("[2001:db8::1]:4242"));
    // a name is never resolved by the numeric lookup
    CHECK(!LookupNumeric("localhost", 1).IsValid());
}

TEST_CASE(netbase_tests, onioncat) {
    // the .onion name and its OnionCat IPv6 form are the same address
    CNetAddr a = IP("5wyqrzbvrdsumnok.onion");
    CNetAddr b = IP("fd87:d87e:eb43:edb1:8e4:3588:e546:35ca");
    CHECK(a == b);
    CHECK(a.IsTor());
    CHECK(a.IsRoutable());
    CHECK_EQ(a.ToStringIP(), std::string("5wyqrzbvrdsumnok.onion"));
}

TEST_CASE(netbase_tests, subnets) {
    // every IPv4 prefix length, written as /n and as a dotted mask, canonicalises to /n with
    // the host bits cleared
    const uint32_t addr = (9u << 24) | (130u << 16) | (77u << 8) | 201u;
    for (int bits = 0; bits <= 32; bits++) {
        const uint32_t m = bits == 0 ? 0 : 0xFFFFFFFFu << (32 - bits);
        const uint32_t netaddr = addr & m;
        const std::string want = strprintf("%u.%u.%u.%u/%d", netaddr >> 24, (netaddr >> 16) & 255, (netaddr >> 8) & 255,
                                           netaddr & 255, bits);
        CSubNet a = Net(strprintf("9.130.77.201/%d", bits)), b = Net("9.130.77.201/" + DottedMask(bits));
        CHECK(a.IsValid());
        CHECK(a == b);
        CHECK_EQ(a.ToString(), want);
        CHECK_EQ(b.ToString(), want);
        CHECK(a.Match(IP("9.130.77.201")));
        // flipping the lowest network bit leaves the subnet (bits > 0)
        if (bits > 0) {
            const uint32_t other = addr ^ (1u << (32 - bits));
            CHECK(!a.Match(IP(strprintf("%u.%u.%u.%u", other >> 24, (other >> 16) & 255, (other >> 8) & 255, other & 255))));
        }
    }
    CHECK(!Net("9.130.77.0/33").IsValid());
    CHECK(!Net("9.130.77.0/-2").IsValid());
    CHECK(Net("2001:db8::/0").IsValid());
    CHECK(Net("2001:db8::/57").IsValid());
    CHECK(Net("2001:db8::/128").IsValid());
    CHECK(!Net("2001:db8::/129").IsValid());
    CHECK(!Net("2001:db8::/-1").IsValid());
    CHECK(!Net("not-a-net").IsValid());
    CHECK(!Net("").IsValid());
    // invalid subnets match nothing
    CHECK(!CSubNet().Match(IP("9.9.9.9")));
    CHECK(!Net("garbage").Match(IP("0.0.0.0")));
    // IPv6 prefixes
    CHECK(Net("2a02:aa:bb::/48").Match(IP("2a02:aa:bb:ffff::1")));
    CHECK(!Net("2a02:aa:bb::/48").Match(IP("2a02:aa:bc::1")));
    CHECK(Net("2a02::1").Match(IP("2a02::1")));
    CHECK(!Net("2a02::1").Match(IP("2a02::2")));
    // documentation addresses (RFC3849) are not valid, so no subnet matches them
    CHECK(!Net("2001:db8::/32").Match(IP("2001:db8::1")));
    CHECK_EQ(Net("2001:db8:1:2:3:4:5:6/ffff:0:0:0:0:0:0:0").ToString(), std::string("2001::/16"));
    CHECK_EQ(Net("2001:db8:1:2:3:4:5:6/0:0:0:0:0:0:0:0").ToString(), std::string("::/0"));
    // ::/0 covers IPv4 too (mapped), 0.0.0.0/0 covers no IPv6 address
    CHECK(Net("::/0").Match(IP("9.8.7.6")));
    CHECK(Net("::/0").Match(IP("2a00::5")));
    CHECK(!Net("0.0.0.0/0").Match(IP("2a00::5")));
    CHECK(Net("::ffff:10.9.8.7").Match(IP("10.9.8.7")));
    // a non-contiguous mask is kept and printed as a mask
    CHECK_EQ(Net("9.130.77.201/255.255.0.255").ToString(), std::string("9.130.0.201/255.255.0.255"));
    CHECK_EQ(Net("2a02:db8:1:3:3:4:5:6/ffff:ffff:ffff:fffe:ffff:ffff:ffff:ff0f").ToString(),
             std::string("2a02:db8:1:2:3:4:5:6/ffff:ffff:ffff:fffe:ffff:ffff:ffff:ff0f"));
    // single-host subnets from an address
    CHECK_EQ(CSubNet(IP("192.0.2.55")).ToString(), std::string("192.0.2.55/32"));
    CHECK(CSubNet(IP("192.0.2.55")).Match(IP("192.0.2.55")));
    CHECK(!CSubNet(IP("192.0.2.55")).Match(IP("192.0.2.56")));
    CHECK_EQ(CSubNet(IP("2a02::9")).ToString(), std::string("2a02::9/128"));
    CHECK_EQ(CSubNet(IP("192.0.2.55"), 16).ToString(), std::string("192.0.0.0/16"));
    CHECK_EQ(CSubNet(IP("192.0.2.55"), 0).ToString(), std::string("0.0.0.0/0"));
}

TEST_CASE(netbase_tests, getgroup) {
    typedef std::vector<unsigned char> V;
    // not routable -> the single "unroutable" group
    for (const char* p : {"127.0.0.9", "192.168.4.4", "169.254.9.9", "0.0.0.0"}) CHECK(IP(p).GetGroup() == V{0});
    // IPv4 /16, also when reached through an IPv6 transition form
    const V g4{NET_IPV4, 93, 184};
    CHECK(IP("93.184.216.34").GetGroup() == g4);
    CHECK(IP("::ffff:0:5db8:d822").GetGroup() == g4);               // RFC6145
    CHECK(IP("64:ff9b::5db8:d822").GetGroup() == g4);               // RFC6052
    CHECK(IP("2002:5db8:d822:1:2:3:4:5").GetGroup() == g4);         // 6to4, RFC3964
    CHECK(IP("2001:0:1:2:3:4:a247:27dd").GetGroup() == g4);         // Teredo, RFC4380 (inverted)
    // Tor: 4 bits of the onion address
    CHECK(IP("fd87:d87e:eb43:f1:8e4:3588:e546:35ca").GetGroup() == (V{NET_TOR, 0x0f}));
    CHECK(IP("fd87:d87e:eb43:edb1:8e4:3588:e546:35ca").GetGroup() == (V{NET_TOR, 239}));
    // Hurricane Electric tunnels: /36 (the partial byte's low bits set); other IPv6: /32
    CHECK(IP("2001:470:1234:5678::1").GetGroup() == (V{NET_IPV6, 0x20, 0x01, 0x04, 0x70, 0x1f}));
    CHECK(IP("2a00:1450:4001:80b::200e").GetGroup() == (V{NET_IPV6, 0x2a, 0x00, 0x14, 0x50}));
}

} // namespace bcp
