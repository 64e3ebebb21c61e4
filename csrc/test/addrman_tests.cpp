// addrman_tests: the peer address manager and the ban list.
// Parity: reference src/test/addrman_tests.cpp (addrman_simple / ports / select / new_collisions /
// tried_collisions / find / create / delete / getaddr, the bucket-placement properties of
// caddrinfo_get_tried_bucket / get_new_bucket: deterministic per key, spread over a bounded set
// of buckets per (source) group) and the ban-list half of DoS_tests.cpp (ban, expiry, unban).
#include "test/unittest.h"

#include "consensus/params.h"
#include "net/addrman.h"
#include "net/net.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <set>

using namespace bcp;

namespace {

CAddress Addr(const std::string& ipport) { return CAddress(LookupNumeric(ipport, 8333), NODE_NETWORK); }
CNetAddr Ip(const std::string& ip) {
    CNetAddr a;
    LookupHost(ip, a, false);
    return a;
}

} // namespace

TEST_CASE(addrman_tests, add_select_good) {
    CAddrMan am;
    // fixed bucket key: with a random one the two ports of 250.1.1.1 share a new-table slot in
    // 1 of 64 runs, and the second Add is then refused (as in the reference, addrman.cpp Add_)
    am.MakeDeterministic();
    CHECK_EQ(am.size(), 0u);
    CHECK(!am.Select().IsValid()); // nothing to select
    const CNetAddr src = Ip("252.2.2.2");
    CHECK(am.Add(Addr("250.1.1.1:8333"), src));
    CHECK_EQ(am.size(), 1u);
    CHECK(am.Select() == Addr("250.1.1.1:8333"));
    // the same address again does not grow the table; another port is another address
    am.Add(Addr("250.1.1.1:8333"), src);
    CHECK_EQ(am.size(), 1u);
    CHECK(am.Add(Addr("250.1.1.1:8334"), src));
    CHECK_EQ(am.size(), 2u);
    // Good() moves an address to the tried table; newOnly selection then skips it
    CHECK_EQ(am.NumTried(), 0u);
    am.Good(LookupNumeric("250.1.1.1:8333", 8333));
    CHECK_EQ(am.NumTried(), 1u);
    CHECK_EQ(am.NumNew(), 1u);
    for (int i = 0; i < 20; i++) CHECK(am.Select(true) == Addr("250.1.1.1:8334"));
    CAddrInfo info;
    CHECK(am.Find(LookupNumeric("250.1.1.1:8333", 8333), &info));
    CHECK(info.fInTried);
    CHECK(!am.Find(LookupNumeric("250.9.9.9:8333", 8333)));
    // non-routable addresses are not kept
    CHECK(!am.Add(Addr("127.0.0.1:8333"), src));
    CHECK(!am.Add(Addr("10.0.0.1:8333"), src));
    CHECK_EQ(am.size(), 2u);
    am.Clear();
    CHECK_EQ(am.size(), 0u);
}

TEST_CASE(addrman_tests, getaddr_bounds) {
    CAddrMan am;
    // 1,000 addresses from many groups, announced by many sources (one source group fills at
    // most 64 new buckets)
    for (int i = 0; i < 1000; i++) {
        CAddress a = Addr(strprintf("250.%d.%d.%d:8333", i % 250, i / 250, 1 + i % 200));
        a.nTime = (uint32_t)GetTime(); // recent (stale addresses are never handed out)
        am.Add(a, Ip(strprintf("252.%d.2.2", i % 200)));
    }
    const size_t n = am.size();
    CHECK(n > 500);
    std::vector<CAddress> v = am.GetAddr();
    CHECK(v.size() <= n * CAddrMan::GETADDR_MAX_PCT / 100 + 1);
    CHECK(v.size() >= n * CAddrMan::GETADDR_MAX_PCT / 100 / 2);
    std::set<std::string> uniq;
    for (const CAddress& a : v) uniq.insert(a.ToString());
    CHECK_EQ(uniq.size(), v.size()); // no duplicates
}

TEST_CASE(addrman_tests, bucket_placement) {
    const uint256 key1 = uint256S("01"), key2 = uint256S("02");
    // tried buckets: deterministic per key; one /16 group lands in at most 8 buckets
    std::set<int> buckets;
    for (int i = 0; i < 255; i++) {
        CAddrInfo info(Addr(strprintf("250.1.1.%d:8333", i)), Ip("250.1.1.1"));
        const int b = info.GetTriedBucket(key1);
        CHECK_EQ(b, info.GetTriedBucket(key1));
        CHECK(b >= 0 && b < CAddrMan::TRIED_BUCKET_COUNT);
        buckets.insert(b);
    }
    CHECK(buckets.size() <= 8u);
    CHECK(buckets.size() > 1u);
    // many groups spread over many tried buckets
    buckets.clear();
    for (int j = 0; j < 255; j++) {
        CAddrInfo info(Addr(strprintf("250.%d.1.1:8333", j)), Ip("250.1.1.1"));
        buckets.insert(info.GetTriedBucket(key1));
    }
    CHECK(buckets.size() > 160u);
    // the salt matters
    int differ = 0;
    for (int j = 0; j < 64; j++) {
        CAddrInfo info(Addr(strprintf("250.%d.2.2:8333", j)), Ip("250.1.1.1"));
        differ += info.GetTriedBucket(key1) != info.GetTriedBucket(key2);
    }
    CHECK(differ > 48);
    // new buckets: addresses announced by one source group occupy at most 64 buckets
    buckets.clear();
    for (int i = 0; i < 4 * 255; i++) {
        CAddrInfo info(Addr(strprintf("250.%d.%d.1:8333", i / 255, i % 255)), Ip("251.4.1.1"));
        const int b = info.GetNewBucket(key1, Ip("251.4.1.1"));
        CHECK(b >= 0 && b < CAddrMan::NEW_BUCKET_COUNT);
        buckets.insert(b);
    }
    CHECK(buckets.size() <= 64u);
    // ... while many source groups spread widely
    buckets.clear();
    for (int s = 0; s < 255; s++) {
        CAddrInfo info(Addr("250.1.1.1:8333"), Ip(strprintf("251.%d.1.1", s)));
        buckets.insert(info.GetNewBucket(key1, Ip(strprintf("251.%d.1.1", s))));
    }
    CHECK(buckets.size() > 8u); // one address, bounded by NEW_BUCKETS_PER_ADDRESS groups of buckets
    // positions within a bucket are in range and differ between new and tried tables
    CAddrInfo info(Addr("250.7.7.7:8333"), Ip("251.1.1.1"));
    const int pn = info.GetBucketPosition(key1, true, 5), pt = info.GetBucketPosition(key1, false, 5);
    CHECK(pn >= 0 && pn < CAddrMan::BUCKET_SIZE && pt >= 0 && pt < CAddrMan::BUCKET_SIZE);
}

TEST_CASE(addrman_tests, terrible_and_persistence) {
    const int64_t now = 1600000000;
    SetMockTime(now);
    CAddrInfo fresh(Addr("250.3.3.3:8333"), Ip("252.2.2.2"));
    fresh.nTime = (uint32_t)now;
    CHECK(!fresh.IsTerrible(now));
    CAddrInfo future = fresh;
    future.nTime = (uint32_t)(now + 20 * 60); // more than 10 minutes in the future
    CHECK(future.IsTerrible(now));
    CAddrInfo stale = fresh;
    stale.nTime = (uint32_t)(now - 31 * 24 * 3600); // older than the 30-day horizon
    CHECK(stale.IsTerrible(now));
    CAddrInfo failing = fresh;
    failing.nAttempts = CAddrMan::RETRIES;
    failing.nLastSuccess = 0;
    CHECK(failing.IsTerrible(now));
    // peers.dat round trip keeps the tables
    CAddrMan am;
    for (int i = 0; i < 200; i++) am.Add(Addr(strprintf("250.%d.9.%d:8333", i % 50, 1 + i)), Ip("252.2.2.2"));
    // bucket positions depend on the table's random key, so an address can lose a collision:
    // move one that made it into the new table to the tried table
    std::string goodAddr;
    for (int i = 0; i < 200 && goodAddr.empty(); i++) {
        const std::string a = strprintf("250.%d.9.%d:8333", i % 50, 1 + i);
        if (am.Find(LookupNumeric(a, 8333))) goodAddr = a;
    }
    REQUIRE(!goodAddr.empty());
    am.Good(LookupNumeric(goodAddr, 8333));
    CHECK_EQ(am.NumTried(), 1u);
    char tmpl[] = "/tmp/bcp_addrman_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    const std::string path = std::string(tmpl) + "/peers.dat";
    const unsigned char magic[4] = {0xfa, 0xbf, 0xb5, 0xda};
    REQUIRE(am.Write(path, magic));
    CAddrMan back;
    REQUIRE(back.Read(path, magic));
    CHECK_EQ(back.size(), am.size());
    CHECK_EQ(back.NumTried(), am.NumTried());
    CAddrInfo found;
    CHECK(back.Find(LookupNumeric(goodAddr, 8333), &found));
    CHECK(found.fInTried);
    // wrong network magic, or a damaged file, is refused
    const unsigned char other[4] = {0xe3, 0xe1, 0xf3, 0xe8};
    CAddrMan wrong;
    CHECK(!wrong.Read(path, other));
    FILE* f = fopen(path.c_str(), "r+b");
    REQUIRE(f != nullptr);
    fseek(f, 40, SEEK_SET);
    fputc(0x55, f);
    fclose(f);
    CAddrMan damaged;
    CHECK(!damaged.Read(path, magic));
    const std::string cmd = std::string("rm -rf '") + tmpl + "'";
    if (system(cmd.c_str()) != 0) {}
    SetMockTime(0);
}

TEST_CASE(addrman_tests, banlist) {
    // DoS_tests ban half: ban, expiry, subnet bans, unban, sweep, persistence
    const int64_t now = 1600000000;
    SetMockTime(now);
    BanMan bm;
    CSubNet one, net;
    REQUIRE(LookupSubNet("250.8.8.8", one));
    REQUIRE(LookupSubNet("251.1.0.0/16", net));
    bm.Ban(one, BanReasonNodeMisbehaving, 3600);
    bm.Ban(net, BanReasonManuallyAdded, 60);
    CHECK(bm.IsBanned(Ip("250.8.8.8")));
    CHECK(!bm.IsBanned(Ip("250.8.8.9")));
    CHECK(bm.IsBanned(Ip("251.1.200.3")));
    CHECK(!bm.IsBanned(Ip("251.2.0.1")));
    // expiry
    SetMockTime(now + 61);
    CHECK(!bm.IsBanned(Ip("251.1.200.3")));
    CHECK(bm.IsBanned(Ip("250.8.8.8")));
    bm.SweepBanned();
    banmap_t m;
    bm.GetBanned(m);
    CHECK_EQ(m.size(), 1u);
    // persistence
    char tmpl[] = "/tmp/bcp_ban_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    const std::string path = std::string(tmpl) + "/banlist.dat";
    const unsigned char magic[4] = {0xfa, 0xbf, 0xb5, 0xda};
    REQUIRE(bm.Write(path, magic));
    BanMan back;
    REQUIRE(back.Read(path, magic));
    CHECK(back.IsBanned(Ip("250.8.8.8")));
    CHECK(back.Unban(one));
    CHECK(!back.IsBanned(Ip("250.8.8.8")));
    CHECK(!back.Unban(one));
    const std::string cmd = std::string("rm -rf '") + tmpl + "'";
    if (system(cmd.c_str()) != 0) {}
    SetMockTime(0);
}

TEST_CASE(addrman_tests, fixed_seeds) {
    // contrib/seeds/generate-seeds.py entries: an IPv4 (v4-mapped) and an IPv6 seed
    const int64_t now = 1600000000;
    SetMockTime(now);
    std::vector<SeedSpec6> seeds(2);
    const unsigned char v4[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff, 1, 2, 3, 4};
    const unsigned char v6[16] = {0x20, 0x01, 0x0d, 0xb8, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
    memcpy(seeds[0].addr, v4, 16);
    seeds[0].port = 8337;
    memcpy(seeds[1].addr, v6, 16);
    seeds[1].port = 18337;
    const std::vector<CAddress> a = ConvertSeed6(seeds);
    REQUIRE(a.size() == 2u);
    CHECK_EQ(a[0].ToStringIPPort(), std::string("1.2.3.4:8337"));
    CHECK(a[0].IsIPv4());
    CHECK_EQ(a[1].ToStringIPPort(), std::string("[2001:db8::1]:18337"));
    for (const CAddress& x : a) {
        CHECK(x.nServices & NODE_NETWORK);
        CHECK((int64_t)x.nTime <= now - 7 * 24 * 3600 && (int64_t)x.nTime > now - 14 * 24 * 3600);
    }
    // the shipped lists (reference: empty) load into the chain parameters
    SelectParams("main");
    CHECK(Params().FixedSeeds().size() < 1000u);
    SetMockTime(0);
}
