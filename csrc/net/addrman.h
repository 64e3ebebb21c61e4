// Peer address manager and ban list.
// Parity: reference src/addrman.{h,cpp} (CAddrMan: 1024 "new" buckets fed by source
// group, 256 "tried" buckets, 64 slots each, salted bucket hashing so an attacker cannot
// choose placement, Add/Good/Attempt/Select/GetAddr/Connected, IsTerrible eviction,
// serialized into peers.dat with a SHA256d checksum by src/addrdb.cpp), and the ban
// list of src/net.cpp/src/addrdb.h (CBanEntry with reason, banlist.dat, SweepBanned).
//
// Design: one mutex-protected table of CAddrInfo indexed by id; bucket slots hold ids.
#pragma once
#include "util/sync.h"
#include "net/netaddress.h"
#include "primitives/uint256.h"

#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace bcp {

class CAddrInfo : public CAddress {
public:
    CAddrInfo() {}
    CAddrInfo(const CAddress& a, const CNetAddr& src) : CAddress(a), source(src) {}
    CNetAddr source;
    int64_t nLastSuccess = 0;
    int nAttempts = 0;
    int nRefCount = 0; // number of new buckets referencing it
    bool fInTried = false;
    int nRandomPos = -1;

    int GetTriedBucket(const uint256& key) const;
    int GetNewBucket(const uint256& key, const CNetAddr& src) const;
    int GetBucketPosition(const uint256& key, bool fNew, int bucket) const;
    bool IsTerrible(int64_t now) const;
    double GetChance(int64_t now) const;

    template <typename S> void Serialize(S& s) const {
        CAddress::Serialize(s);
        source.Serialize(s);
        ::bcp::Serialize(s, nLastSuccess);
        ::bcp::Serialize(s, nAttempts);
    }
    template <typename S> void Unserialize(S& s) {
        CAddress::Unserialize(s);
        source.Unserialize(s);
        ::bcp::Unserialize(s, nLastSuccess);
        ::bcp::Unserialize(s, nAttempts);
    }
};

class CAddrMan {
public:
    static const int TRIED_BUCKET_COUNT = 256;
    static const int NEW_BUCKET_COUNT = 1024;
    static const int BUCKET_SIZE = 64;
    static const int NEW_BUCKETS_PER_ADDRESS = 8;
    static const int HORIZON_DAYS = 30;
    static const int RETRIES = 3;
    static const int MAX_FAILURES = 10;
    static const int MIN_FAIL_DAYS = 7;
    static const int GETADDR_MAX_PCT = 23;
    static const int GETADDR_MAX = 2500;

    CAddrMan();
    void Clear();
    size_t size() const;
    bool Add(const CAddress& addr, const CNetAddr& source, int64_t nTimePenalty = 0);
    bool Add(const std::vector<CAddress>& v, const CNetAddr& source, int64_t nTimePenalty = 0);
    void Good(const CService& addr, int64_t nTime = 0);
    void Attempt(const CService& addr, bool fCountFailure, int64_t nTime = 0);
    CAddrInfo Select(bool newOnly = false);
    std::vector<CAddress> GetAddr();
    void Connected(const CService& addr, int64_t nTime = 0);
    void SetServices(const CService& addr, uint64_t services);
    bool Find(const CService& addr, CAddrInfo* out = nullptr) const;
    size_t NumTried() const;
    size_t NumNew() const;
    // Tests: a fixed (null) bucket key, so placements repeat run to run (the reference's
    // CAddrManSerializationMock::MakeDeterministic, src/test/net_tests.cpp:23)
    void MakeDeterministic() { nKey.SetNull(); }

    // peers.dat: magic + version + key + entries + SHA256d checksum
    bool Write(const std::string& path, const unsigned char* magic) const;
    bool Read(const std::string& path, const unsigned char* magic);

private:
    int Id(const CService& addr) const;
    int Create(const CAddress& addr, const CNetAddr& src);
    void Delete(int id);
    void ClearNew(int bucket, int pos);
    void MakeTried(int id);
    void SwapRandom(int a, int b);

    mutable CCriticalSection cs{"addrman.cs"};
    uint256 nKey;
    std::map<int, CAddrInfo> mapInfo;
    std::map<std::vector<unsigned char>, int> mapAddr;
    std::vector<int> vRandom;
    int nIdCount = 0;
    int nTried = 0, nNew = 0;
    std::vector<int> vvTried; // TRIED_BUCKET_COUNT * BUCKET_SIZE, -1 empty
    std::vector<int> vvNew;
    int64_t nLastGood = 1;
};

enum BanReason { BanReasonUnknown = 0, BanReasonNodeMisbehaving = 1, BanReasonManuallyAdded = 2 };

struct CBanEntry {
    int32_t nVersion = 1;
    int64_t nCreateTime = 0;
    int64_t nBanUntil = 0;
    uint8_t banReason = BanReasonUnknown;
    std::string BanReasonToString() const {
        return banReason == BanReasonNodeMisbehaving ? "node misbehaving"
               : banReason == BanReasonManuallyAdded ? "manually added"
                                                      : "unknown";
    }
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, nCreateTime);
        ::bcp::Serialize(s, nBanUntil);
        ::bcp::Serialize(s, banReason);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, nCreateTime);
        ::bcp::Unserialize(s, nBanUntil);
        ::bcp::Unserialize(s, banReason);
    }
};
typedef std::map<CSubNet, CBanEntry> banmap_t;

class BanMan {
public:
    void Ban(const CSubNet& sub, BanReason reason, int64_t bantime = 0, bool sinceUnixEpoch = false);
    bool Unban(const CSubNet& sub);
    bool IsBanned(const CNetAddr& ip);
    bool IsBanned(const CSubNet& sub);
    void GetBanned(banmap_t& out);
    void SetBanned(const banmap_t& m);
    void ClearBanned();
    void SweepBanned();
    bool Dirty() const { return dirty; }
    bool Write(const std::string& path, const unsigned char* magic);
    bool Read(const std::string& path, const unsigned char* magic);

private:
    std::mutex cs;
    banmap_t banned;
    bool dirty = false;
};

} // namespace bcp
