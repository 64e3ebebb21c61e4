#include "net/addrman.h"
#include "net/protocol.h"
#include "crypto/hashes.h"
#include "keys/key.h"
#include "util/util.h"

#include <cmath>

namespace bcp {

static uint64_t HashKeyed(const uint256& key, const std::vector<unsigned char>& data) {
    HashWriter hw;
    hw.write((const char*)key.begin(), 32);
    hw.write((const char*)data.data(), data.size());
    const uint256 h = hw.GetHash();
    uint64_t r;
    memcpy(&r, h.begin(), 8);
    return r;
}

static std::vector<unsigned char> Cat(std::vector<unsigned char> a, const std::vector<unsigned char>& b) {
    a.insert(a.end(), b.begin(), b.end());
    return a;
}
static std::vector<unsigned char> U64(uint64_t v) {
    std::vector<unsigned char> r(8);
    memcpy(r.data(), &v, 8);
    return r;
}

// Tried placement: the address picks one of 8 buckets within its /16 group.
int CAddrInfo::GetTriedBucket(const uint256& key) const {
    const uint64_t h1 = HashKeyed(key, GetKey()) % 8;
    const uint64_t h2 = HashKeyed(key, Cat(GetGroup(), U64(h1))) % CAddrMan::TRIED_BUCKET_COUNT;
    return (int)h2;
}

// New placement: the source group picks 64 candidate buckets, the address group one of them.
int CAddrInfo::GetNewBucket(const uint256& key, const CNetAddr& src) const {
    const std::vector<unsigned char> srcGroup = src.GetGroup();
    const uint64_t h1 = HashKeyed(key, Cat(GetGroup(), srcGroup)) % 64;
    const uint64_t h2 = HashKeyed(key, Cat(srcGroup, U64(h1))) % CAddrMan::NEW_BUCKET_COUNT;
    return (int)h2;
}

int CAddrInfo::GetBucketPosition(const uint256& key, bool fNew, int bucket) const {
    std::vector<unsigned char> d{(unsigned char)(fNew ? 'N' : 'K')};
    d = Cat(d, U64((uint64_t)bucket));
    d = Cat(d, GetKey());
    return (int)(HashKeyed(key, d) % CAddrMan::BUCKET_SIZE);
}

bool CAddrInfo::IsTerrible(int64_t now) const {
    if (nLastTry && nLastTry >= now - 60) return false;                  // tried in the last minute
    if (nTime > now + 10 * 60) return true;                              // came in a flying DeLorean
    if (nTime == 0 || now - nTime > CAddrMan::HORIZON_DAYS * 24 * 60 * 60) return true;
    if (nLastSuccess == 0 && nAttempts >= CAddrMan::RETRIES) return true; // never succeeded
    if (now - nLastSuccess > CAddrMan::MIN_FAIL_DAYS * 24 * 60 * 60 && nAttempts >= CAddrMan::MAX_FAILURES) return true;
    return false;
}

double CAddrInfo::GetChance(int64_t now) const {
    double chance = 1.0;
    const int64_t sinceLastTry = std::max<int64_t>(now - nLastTry, 0);
    if (sinceLastTry < 60 * 10) chance *= 0.01;
    chance *= std::pow(0.66, std::min(nAttempts, 8));
    return chance;
}

CAddrMan::CAddrMan() { Clear(); }

void CAddrMan::Clear() {
    std::lock_guard<CCriticalSection> l(cs);
    nKey = GetRandHash();
    mapInfo.clear();
    mapAddr.clear();
    vRandom.clear();
    nIdCount = nTried = nNew = 0;
    vvTried.assign(TRIED_BUCKET_COUNT * BUCKET_SIZE, -1);
    vvNew.assign(NEW_BUCKET_COUNT * BUCKET_SIZE, -1);
    nLastGood = 1;
}

size_t CAddrMan::size() const {
    std::lock_guard<CCriticalSection> l(cs);
    return vRandom.size();
}
size_t CAddrMan::NumTried() const {
    std::lock_guard<CCriticalSection> l(cs);
    return nTried;
}
size_t CAddrMan::NumNew() const {
    std::lock_guard<CCriticalSection> l(cs);
    return nNew;
}

int CAddrMan::Id(const CService& addr) const {
    auto it = mapAddr.find(addr.GetKey());
    return it == mapAddr.end() ? -1 : it->second;
}

bool CAddrMan::Find(const CService& addr, CAddrInfo* out) const {
    std::lock_guard<CCriticalSection> l(cs);
    const int id = Id(addr);
    if (id < 0) return false;
    if (out) *out = mapInfo.at(id);
    return true;
}

int CAddrMan::Create(const CAddress& addr, const CNetAddr& src) {
    const int id = nIdCount++;
    CAddrInfo& info = mapInfo[id];
    info = CAddrInfo(addr, src);
    mapAddr[addr.GetKey()] = id;
    info.nRandomPos = (int)vRandom.size();
    vRandom.push_back(id);
    return id;
}

void CAddrMan::SwapRandom(int a, int b) {
    if (a == b) return;
    const int ida = vRandom[a], idb = vRandom[b];
    mapInfo[ida].nRandomPos = b;
    mapInfo[idb].nRandomPos = a;
    vRandom[a] = idb;
    vRandom[b] = ida;
}

void CAddrMan::Delete(int id) {
    CAddrInfo& info = mapInfo[id];
    SwapRandom(info.nRandomPos, (int)vRandom.size() - 1);
    vRandom.pop_back();
    mapAddr.erase(info.GetKey());
    mapInfo.erase(id);
    nNew--;
}

void CAddrMan::ClearNew(int bucket, int pos) {
    int& slot = vvNew[bucket * BUCKET_SIZE + pos];
    if (slot == -1) return;
    const int id = slot;
    CAddrInfo& info = mapInfo[id];
    info.nRefCount--;
    slot = -1;
    if (info.nRefCount == 0) Delete(id);
}

void CAddrMan::MakeTried(int id) {
    CAddrInfo& info = mapInfo[id];
    // remove from every new bucket
    for (int b = 0; b < NEW_BUCKET_COUNT; b++) {
        const int pos = info.GetBucketPosition(nKey, true, b);
        if (vvNew[b * BUCKET_SIZE + pos] == id) {
            vvNew[b * BUCKET_SIZE + pos] = -1;
            info.nRefCount--;
        }
    }
    nNew--;
    const int kb = info.GetTriedBucket(nKey);
    const int kpos = info.GetBucketPosition(nKey, false, kb);
    int& slot = vvTried[kb * BUCKET_SIZE + kpos];
    if (slot != -1) {
        // evict the occupant back to the new table
        const int old = slot;
        CAddrInfo& oinfo = mapInfo[old];
        oinfo.fInTried = false;
        slot = -1;
        nTried--;
        const int nb = oinfo.GetNewBucket(nKey, oinfo.source);
        const int npos = oinfo.GetBucketPosition(nKey, true, nb);
        ClearNew(nb, npos);
        vvNew[nb * BUCKET_SIZE + npos] = old;
        oinfo.nRefCount = 1;
        nNew++;
    }
    slot = id;
    nTried++;
    info.fInTried = true;
}

bool CAddrMan::Add(const CAddress& addr, const CNetAddr& source, int64_t nTimePenalty) {
    std::lock_guard<CCriticalSection> l(cs);
    if (!addr.IsRoutable()) return false;
    const int64_t now = GetAdjustedTime();
    if (addr == source) nTimePenalty = 0;
    int id = Id(addr);
    bool fNew = false;
    if (id >= 0) {
        CAddrInfo& info = mapInfo[id];
        // periodically refresh nTime, merge services
        const bool fCurrentlyOnline = now - addr.nTime < 24 * 60 * 60;
        const int64_t update = fCurrentlyOnline ? 60 * 60 : 24 * 60 * 60;
        if (addr.nTime && (!info.nTime || info.nTime < addr.nTime - update - nTimePenalty))
            info.nTime = (uint32_t)std::max<int64_t>(0, addr.nTime - nTimePenalty);
        info.nServices |= addr.nServices;
        if (!addr.nTime || (info.nTime && addr.nTime <= info.nTime)) return false;
        if (info.fInTried) return false;
        if (info.nRefCount == NEW_BUCKETS_PER_ADDRESS) return false;
        // stochastic: each extra reference is exponentially less likely
        int factor = 1;
        for (int n = 0; n < info.nRefCount; n++) factor *= 2;
        if (factor > 1 && GetRandInt(factor) != 0) return false;
    } else {
        CAddress a = addr;
        a.nTime = (uint32_t)std::max<int64_t>(0, (int64_t)a.nTime - nTimePenalty);
        id = Create(a, source);
        nNew++;
        fNew = true;
    }
    CAddrInfo& info = mapInfo[id];
    const int b = info.GetNewBucket(nKey, source);
    const int pos = info.GetBucketPosition(nKey, true, b);
    int& slot = vvNew[b * BUCKET_SIZE + pos];
    if (slot != id) {
        bool fInsert = slot == -1;
        if (!fInsert) {
            CAddrInfo& existing = mapInfo[slot];
            if (existing.IsTerrible(now) || (existing.nRefCount > 1 && info.nRefCount == 0)) fInsert = true;
        }
        if (fInsert) {
            ClearNew(b, pos);
            info.nRefCount++;
            vvNew[b * BUCKET_SIZE + pos] = id;
        } else if (info.nRefCount == 0) {
            Delete(id);
            return false;
        }
    }
    return fNew;
}

bool CAddrMan::Add(const std::vector<CAddress>& v, const CNetAddr& source, int64_t nTimePenalty) {
    int added = 0;
    for (const CAddress& a : v) added += Add(a, source, nTimePenalty) ? 1 : 0;
    if (added) LogPrintCat(BCLog::ADDRMAN, "Added %d addresses from %s: %zu tried, %zu new\n", added,
                           source.ToString().c_str(), NumTried(), NumNew());
    return added > 0;
}

void CAddrMan::Good(const CService& addr, int64_t nTime) {
    std::lock_guard<CCriticalSection> l(cs);
    if (!nTime) nTime = GetAdjustedTime();
    nLastGood = nTime;
    const int id = Id(addr);
    if (id < 0) return;
    CAddrInfo& info = mapInfo[id];
    if ((CService&)info != addr) return;
    info.nLastSuccess = nTime;
    info.nLastTry = nTime;
    info.nAttempts = 0;
    if (info.fInTried) return;
    MakeTried(id);
}

void CAddrMan::Attempt(const CService& addr, bool fCountFailure, int64_t nTime) {
    std::lock_guard<CCriticalSection> l(cs);
    if (!nTime) nTime = GetAdjustedTime();
    const int id = Id(addr);
    if (id < 0) return;
    CAddrInfo& info = mapInfo[id];
    info.nLastTry = nTime;
    if (fCountFailure && info.nLastTry >= nLastGood) info.nAttempts++;
    if (fCountFailure) info.nAttempts = std::max(info.nAttempts, 1);
}

CAddrInfo CAddrMan::Select(bool newOnly) {
    std::lock_guard<CCriticalSection> l(cs);
    if (vRandom.empty()) return CAddrInfo();
    if (newOnly && nNew == 0) return CAddrInfo();
    const int64_t now = GetAdjustedTime();
    const bool useTried = !newOnly && nTried > 0 && (nNew == 0 || GetRandInt(2) == 0);
    const std::vector<int>& table = useTried ? vvTried : vvNew;
    const int nBuckets = useTried ? TRIED_BUCKET_COUNT : NEW_BUCKET_COUNT;
    double factor = 1.0;
    for (int iter = 0; iter < 100000; iter++) {
        const int b = GetRandInt(nBuckets);
        int pos = GetRandInt(BUCKET_SIZE);
        int k = 0;
        while (k < BUCKET_SIZE && table[b * BUCKET_SIZE + (pos + k) % BUCKET_SIZE] == -1) k++;
        if (k == BUCKET_SIZE) continue;
        const int id = table[b * BUCKET_SIZE + (pos + k) % BUCKET_SIZE];
        const CAddrInfo& info = mapInfo[id];
        if (GetRandInt(1 << 30) < factor * info.GetChance(now) * (1 << 30)) return info;
        factor *= 1.2;
    }
    return mapInfo[vRandom[GetRandInt((int)vRandom.size())]];
}

std::vector<CAddress> CAddrMan::GetAddr() {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<CAddress> out;
    size_t n = GETADDR_MAX_PCT * vRandom.size() / 100;
    n = std::min<size_t>(n, GETADDR_MAX);
    const int64_t now = GetAdjustedTime();
    for (size_t i = 0; i < vRandom.size() && out.size() < n; i++) {
        const int r = (int)(GetRand(vRandom.size() - i) + i);
        SwapRandom((int)i, r);
        const CAddrInfo& info = mapInfo[vRandom[i]];
        if (!info.IsTerrible(now)) out.push_back(info);
    }
    return out;
}

void CAddrMan::Connected(const CService& addr, int64_t nTime) {
    std::lock_guard<CCriticalSection> l(cs);
    if (!nTime) nTime = GetAdjustedTime();
    const int id = Id(addr);
    if (id < 0) return;
    CAddrInfo& info = mapInfo[id];
    if (nTime - info.nTime > 20 * 60) info.nTime = (uint32_t)nTime;
}

void CAddrMan::SetServices(const CService& addr, uint64_t services) {
    std::lock_guard<CCriticalSection> l(cs);
    const int id = Id(addr);
    if (id >= 0) mapInfo[id].nServices = services;
}

static const uint8_t ADDRMAN_FORMAT = 1;

bool CAddrMan::Write(const std::string& path, const unsigned char* magic) const {
    std::vector<unsigned char> payload;
    {
        std::lock_guard<CCriticalSection> l(cs);
        VectorWriter w(payload, SER_DISK, CLIENT_VERSION);
        w.write((const char*)magic, 4);
        w << ADDRMAN_FORMAT << nKey;
        // entries: tried flag + info; new-bucket placement is recomputed on load
        const uint32_t n = (uint32_t)mapInfo.size();
        w << n;
        for (const auto& kv : mapInfo) {
            const uint8_t tried = kv.second.fInTried;
            w << tried << kv.second;
        }
    }
    const uint256 sum = Hash256(payload);
    payload.insert(payload.end(), sum.begin(), sum.end());
    const std::string tmp = path + ".new";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(payload.data(), 1, payload.size(), f) == payload.size();
    FileCommit(f);
    fclose(f);
    return ok && RenameOver(tmp, path);
}

bool CAddrMan::Read(const std::string& path, const unsigned char* magic) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<unsigned char> data;
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    if (data.size() < 4 + 1 + 32 + 4 + 32) return false;
    const uint256 sum = Hash256(data.data(), data.size() - 32);
    if (memcmp(sum.begin(), data.data() + data.size() - 32, 32) != 0) return error("%s: checksum mismatch", __func__);
    if (memcmp(data.data(), magic, 4) != 0) return error("%s: invalid network magic", __func__);
    try {
        SpanReader r(data.data() + 4, data.size() - 36, SER_DISK, CLIENT_VERSION);
        uint8_t fmt;
        uint256 key;
        uint32_t count;
        r >> fmt >> key >> count;
        if (fmt != ADDRMAN_FORMAT) return false;
        std::lock_guard<CCriticalSection> l(cs);
        Clear();
        nKey = key;
        for (uint32_t i = 0; i < count; i++) {
            uint8_t tried;
            CAddrInfo info;
            r >> tried >> info;
            if (Id(info) >= 0) continue;
            const int id = Create(info, info.source);
            CAddrInfo& in = mapInfo[id];
            in.nLastSuccess = info.nLastSuccess;
            in.nAttempts = info.nAttempts;
            nNew++;
            const int b = in.GetNewBucket(nKey, in.source);
            const int pos = in.GetBucketPosition(nKey, true, b);
            if (vvNew[b * BUCKET_SIZE + pos] == -1) {
                vvNew[b * BUCKET_SIZE + pos] = id;
                in.nRefCount = 1;
            }
            if (tried && in.nRefCount) {
                const int kb = in.GetTriedBucket(nKey);
                const int kpos = in.GetBucketPosition(nKey, false, kb);
                if (vvTried[kb * BUCKET_SIZE + kpos] == -1) MakeTried(id);
            }
            if (!in.nRefCount && !in.fInTried) Delete(id);
        }
    } catch (const std::exception& e) {
        // a file that claims more than it holds leaves no half-loaded table behind
        // (reference addrdb.cpp CAddrDB::Read -> addr.Clear())
        std::lock_guard<CCriticalSection> l(cs);
        Clear();
        return error("%s: deserialize error: %s", __func__, e.what());
    }
    return true;
}

// ------------------------------------------------------------------ ban list
void BanMan::Ban(const CSubNet& sub, BanReason reason, int64_t bantime, bool sinceUnixEpoch) {
    CBanEntry e;
    e.nCreateTime = GetTime();
    e.banReason = (uint8_t)reason;
    if (bantime <= 0) bantime = gArgs.GetArg("-bantime", DEFAULT_MISBEHAVING_BANTIME);
    e.nBanUntil = (sinceUnixEpoch ? 0 : GetTime()) + bantime;
    std::lock_guard<std::mutex> l(cs);
    if (banned[sub].nBanUntil < e.nBanUntil) {
        banned[sub] = e;
        dirty = true;
    }
}

bool BanMan::Unban(const CSubNet& sub) {
    std::lock_guard<std::mutex> l(cs);
    if (!banned.erase(sub)) return false;
    dirty = true;
    return true;
}

bool BanMan::IsBanned(const CNetAddr& ip) {
    std::lock_guard<std::mutex> l(cs);
    const int64_t now = GetTime();
    for (const auto& kv : banned)
        if (kv.first.Match(ip) && now < kv.second.nBanUntil) return true;
    return false;
}

bool BanMan::IsBanned(const CSubNet& sub) {
    std::lock_guard<std::mutex> l(cs);
    auto it = banned.find(sub);
    return it != banned.end() && GetTime() < it->second.nBanUntil;
}

void BanMan::GetBanned(banmap_t& out) {
    SweepBanned();
    std::lock_guard<std::mutex> l(cs);
    out = banned;
}

void BanMan::SetBanned(const banmap_t& m) {
    std::lock_guard<std::mutex> l(cs);
    banned = m;
    dirty = true;
}

void BanMan::ClearBanned() {
    std::lock_guard<std::mutex> l(cs);
    banned.clear();
    dirty = true;
}

void BanMan::SweepBanned() {
    std::lock_guard<std::mutex> l(cs);
    const int64_t now = GetTime();
    for (auto it = banned.begin(); it != banned.end();) {
        if (now > it->second.nBanUntil) {
            it = banned.erase(it);
            dirty = true;
        } else {
            ++it;
        }
    }
}

bool BanMan::Write(const std::string& path, const unsigned char* magic) {
    SweepBanned();
    std::vector<unsigned char> payload;
    {
        std::lock_guard<std::mutex> l(cs);
        VectorWriter w(payload, SER_DISK, CLIENT_VERSION);
        w.write((const char*)magic, 4);
        w << banned;
        dirty = false;
    }
    const uint256 sum = Hash256(payload);
    payload.insert(payload.end(), sum.begin(), sum.end());
    const std::string tmp = path + ".new";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(payload.data(), 1, payload.size(), f) == payload.size();
    FileCommit(f);
    fclose(f);
    return ok && RenameOver(tmp, path);
}

bool BanMan::Read(const std::string& path, const unsigned char* magic) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<unsigned char> data;
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    if (data.size() < 36) return false;
    const uint256 sum = Hash256(data.data(), data.size() - 32);
    if (memcmp(sum.begin(), data.data() + data.size() - 32, 32) != 0) return false;
    if (memcmp(data.data(), magic, 4) != 0) return false;
    try {
        SpanReader r(data.data() + 4, data.size() - 36, SER_DISK, CLIENT_VERSION);
        banmap_t m;
        r >> m;
        std::lock_guard<std::mutex> l(cs);
        banned = m;
        dirty = false;
    } catch (const std::exception&) {
        return false;
    }
    SweepBanned();
    return true;
}

} // namespace bcp
