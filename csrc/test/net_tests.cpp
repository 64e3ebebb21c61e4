// net_tests: peers.dat reads (intact and corrupted), CNode defaults, the EB sub-version and the
// user agent's length cap.
// Parity: reference src/test/net_tests.cpp (caddrdb_read, caddrdb_read_corrupted,
// cnode_simple_test, test_getSubVersionEB, test_userAgentLength). The corrupted file here keeps
// a valid checksum (this format has one), so only the count/entries mismatch is being tested.
#include "test/unittest.h"

#include "crypto/hashes.h"
#include "net/addrman.h"
#include "net/net.h"
#include "net/protocol.h"
#include "node/miner.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <cstdio>
#include <cstdlib>

using namespace bcp;

namespace {

CAddress Addr(const std::string& ipport) { return CAddress(LookupNumeric(ipport, 8333), NODE_NETWORK); }
CNetAddr Ip(const std::string& ip) {
    CNetAddr a;
    LookupHost(ip, a, false);
    return a;
}
const unsigned char MAGIC[4] = {0xe3, 0xe1, 0xf3, 0xe8};

struct TmpDir {
    std::string path;
    TmpDir() {
        char tmpl[] = "/tmp/bcp_net_tests_XXXXXX";
        if (!mkdtemp(tmpl)) throw std::runtime_error("mkdtemp");
        path = tmpl;
    }
    ~TmpDir() {
        const std::string cmd = "rm -rf '" + path + "'";
        if (system(cmd.c_str()) != 0) {}
    }
};

void WriteFile(const std::string& p, const std::vector<unsigned char>& v) {
    FILE* f = fopen(p.c_str(), "wb");
    if (!f || fwrite(v.data(), 1, v.size(), f) != v.size()) throw std::runtime_error("write " + p);
    fclose(f);
}

} // namespace

TEST_CASE(net_tests, caddrdb_read) {
    TmpDir d;
    CAddrMan am;
    am.MakeDeterministic();
    const CNetAddr source = Ip("252.5.1.1");
    for (const char* a : {"250.7.1.1:8337", "250.7.2.2:9999", "250.7.3.3:9999"}) CHECK(am.Add(Addr(a), source));
    CHECK_EQ(am.size(), (size_t)3);
    const std::string path = d.path + "/peers.dat";
    REQUIRE(am.Write(path, MAGIC));
    CAddrMan back;
    CHECK_EQ(back.size(), (size_t)0);
    CHECK(back.Read(path, MAGIC));
    CHECK_EQ(back.size(), (size_t)3);
    for (const char* a : {"250.7.1.1:8337", "250.7.2.2:9999", "250.7.3.3:9999"}) CHECK(back.Find(LookupNumeric(a, 8333)));
}

TEST_CASE(net_tests, caddrdb_read_corrupted) {
    // a well-formed file (magic, format, key, checksum) that claims 20 entries and holds one
    TmpDir d;
    std::vector<unsigned char> payload;
    {
        VectorWriter w(payload, SER_DISK, CLIENT_VERSION);
        w.write((const char*)MAGIC, 4);
        w << (uint8_t)1 << uint256() << (uint32_t)20;
        CAddrInfo info(Addr("252.1.1.1:7777"), Ip("252.2.2.2"));
        w << (uint8_t)0 << info;
    }
    const uint256 sum = Hash256(payload);
    payload.insert(payload.end(), sum.begin(), sum.end());
    const std::string path = d.path + "/peers.dat";
    WriteFile(path, payload);
    // the read fails and leaves nothing behind (the entry it did decode is dropped too)
    CAddrMan am;
    CHECK(am.Add(Addr("250.1.1.1:8333"), Ip("252.5.1.1"))); // whatever was there before goes as well
    CHECK(!am.Read(path, MAGIC));
    CHECK_EQ(am.size(), (size_t)0);
    // and the same bytes with an honest count load
    payload.resize(payload.size() - 32);
    payload[4 + 1 + 32] = 1;
    const uint256 sum2 = Hash256(payload);
    payload.insert(payload.end(), sum2.begin(), sum2.end());
    WriteFile(path, payload);
    CAddrMan ok;
    CHECK(ok.Read(path, MAGIC));
    CHECK_EQ(ok.size(), (size_t)1);
}

TEST_CASE(net_tests, cnode_simple) {
    const CAddress addr(LookupNumeric("160.176.192.1:7777", 7777), NODE_NETWORK);
    CNode out(0, NODE_NETWORK, 0, -1, addr, 0, 0, "", false);
    CHECK(!out.fInbound);
    CHECK(!out.fFeeler);
    CNode in(1, NODE_NETWORK, 0, -1, addr, 1, 1, "", true);
    CHECK(in.fInbound);
    CHECK(!in.fFeeler);
    CHECK_EQ((long long)in.GetId(), 1LL);
}

TEST_CASE(net_tests, sub_version_eb) {
    CHECK_EQ(GetSubVersionEB(13800000000ULL), std::string("13800.0"));
    CHECK_EQ(GetSubVersionEB(3800000000ULL), std::string("3800.0"));
    CHECK_EQ(GetSubVersionEB(14000000), std::string("14.0"));
    CHECK_EQ(GetSubVersionEB(1540000), std::string("1.5"));
    CHECK_EQ(GetSubVersionEB(1560000), std::string("1.5")); // floored, not rounded
    CHECK_EQ(GetSubVersionEB(210000), std::string("0.2"));
    CHECK_EQ(GetSubVersionEB(10000), std::string("0.0"));
    CHECK_EQ(GetSubVersionEB(0), std::string("0.0"));
}

TEST_CASE(net_tests, user_agent_length) {
    std::string very;
    for (int i = 0; i < 62; i++) very += "very ";
    very += "long comment";
    gArgs.ForceSetArg("-uacomment", very);
    const std::string ua = UserAgent(8000000);
    gArgs.ForceSetArg("-uacomment", "");
    gArgs.ClearArg("-uacomment");
    // cut to the limit and closed again: "/<name>:<version>(EB8.0; very very ... v)/"
    CHECK_EQ(ua.size(), (size_t)MAX_SUBVERSION_LENGTH);
    const std::string head = std::string("/") + CLIENT_NAME + ":";
    CHECK_EQ(ua.compare(0, head.size(), head), 0);
    CHECK(ua.find("(EB8.0; very very") != std::string::npos);
    CHECK_EQ(ua.substr(ua.size() - 3), std::string("v)/"));
    // a short comment is kept whole
    gArgs.ForceSetArg("-uacomment", "short");
    const std::string ua2 = UserAgent(8000000);
    gArgs.ClearArg("-uacomment");
    CHECK(ua2.find("(EB8.0; short)/") != std::string::npos);
    CHECK(UserAgent(8000000).find("(EB8.0)/") != std::string::npos);
}
