#include "node/kvstore.h"

#include <array>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <stdexcept>
#include <sys/stat.h>
#include <unistd.h>

namespace bcp {

namespace {
const uint32_t BATCH_MAGIC = 0xB7C0DB01;
const uint8_t OP_PUT = 1, OP_DEL = 2;

uint32_t Crc32c(const unsigned char* p, size_t n) {
    static const std::array<uint32_t, 256> table = [] {
        std::array<uint32_t, 256> t{};
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
            t[i] = c;
        }
        return t;
    }();
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

void PutVar(std::string& out, uint64_t v) {
    while (v >= 0x80) {
        out.push_back((char)(v | 0x80));
        v >>= 7;
    }
    out.push_back((char)v);
}
bool GetVar(const unsigned char*& p, const unsigned char* end, uint64_t& v) {
    v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
        if (p >= end) return false;
        const unsigned char b = *p++;
        v |= (uint64_t)(b & 0x7f) << shift;
        if (!(b & 0x80)) return true;
    }
    return false;
}
bool WriteAll(int fd, const void* data, size_t n) {
    const char* p = (const char*)data;
    while (n) {
        ssize_t w = ::write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        n -= (size_t)w;
    }
    return true;
}
bool PreadAll(int fd, void* data, size_t n, uint64_t off) {
    char* p = (char*)data;
    while (n) {
        ssize_t r = ::pread(fd, p, n, (off_t)off);
        if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            return false;
        }
        p += r;
        n -= (size_t)r;
        off += (uint64_t)r;
    }
    return true;
}
void MkdirP(const std::string& path) {
    std::string cur;
    for (size_t i = 0; i < path.size(); i++) {
        cur.push_back(path[i]);
        if (path[i] == '/' || i + 1 == path.size()) ::mkdir(cur.c_str(), 0700);
    }
}
} // namespace

KVStore::KVStore(const std::string& path, bool memory_only, bool wipe) : dir(path), memOnly(memory_only) {
    if (memOnly) return;
    MkdirP(dir);
    logPath = dir + "/kv.log";
    if (wipe) ::unlink(logPath.c_str());
    fd = ::open(logPath.c_str(), O_RDWR | O_CREAT, 0600);
    if (fd < 0) throw std::runtime_error("KVStore: cannot open " + logPath + ": " + strerror(errno));
    if (!Replay()) throw std::runtime_error("KVStore: corrupt log " + logPath);
}

KVStore::~KVStore() {
    if (fd >= 0) {
        ::fsync(fd);
        ::close(fd);
    }
}

// Rebuild the index from the log; a torn/corrupt tail is truncated.
bool KVStore::Replay() {
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    const uint64_t size = (uint64_t)st.st_size;
    uint64_t off = 0;
    std::vector<unsigned char> buf;
    while (off + 12 <= size) {
        unsigned char hdr[12];
        if (!PreadAll(fd, hdr, 12, off)) break;
        uint32_t magic, len, crc;
        memcpy(&magic, hdr, 4);
        memcpy(&len, hdr + 4, 4);
        memcpy(&crc, hdr + 8, 4);
        if (magic != BATCH_MAGIC || off + 12 + len > size) break;
        buf.resize(len);
        if (!PreadAll(fd, buf.data(), len, off + 12)) break;
        if (Crc32c(buf.data(), len) != crc) break;
        const unsigned char* p = buf.data();
        const unsigned char* end = p + len;
        bool ok = true;
        while (p < end) {
            const uint8_t op = *p++;
            uint64_t klen, vlen = 0;
            if (!GetVar(p, end, klen) || (uint64_t)(end - p) < klen) {
                ok = false;
                break;
            }
            std::string key((const char*)p, klen);
            p += klen;
            if (op == OP_PUT) {
                if (!GetVar(p, end, vlen) || (uint64_t)(end - p) < vlen) {
                    ok = false;
                    break;
                }
                const uint64_t voff = off + 12 + (uint64_t)(p - buf.data());
                auto it = index.find(key);
                if (it != index.end()) liveBytes -= it->second.len + it->first.size();
                index[key] = Loc{voff, (uint32_t)vlen};
                liveBytes += vlen + key.size();
                p += vlen;
            } else if (op == OP_DEL) {
                auto it = index.find(key);
                if (it != index.end()) {
                    liveBytes -= it->second.len + it->first.size();
                    index.erase(it);
                }
            } else {
                ok = false;
                break;
            }
        }
        if (!ok) break;
        off += 12 + len;
    }
    if (off != size) {
        if (ftruncate(fd, (off_t)off) != 0) return false;
    }
    logSize = off;
    return true;
}

std::map<std::string, std::string> KVStore::Salvage(const std::string& dir, uint64_t* skipped) {
    std::map<std::string, std::string> out;
    if (skipped) *skipped = 0;
    const std::string path = dir + "/kv.log";
    const int f = ::open(path.c_str(), O_RDONLY);
    if (f < 0) return out;
    struct stat st;
    if (fstat(f, &st) != 0) {
        ::close(f);
        return out;
    }
    std::vector<unsigned char> log((size_t)st.st_size);
    const bool read_ok = log.empty() || PreadAll(f, log.data(), log.size(), 0);
    ::close(f);
    if (!read_ok) return out;
    size_t off = 0;
    while (off + 12 <= log.size()) {
        uint32_t magic, len, crc;
        memcpy(&magic, &log[off], 4);
        memcpy(&len, &log[off + 4], 4);
        memcpy(&crc, &log[off + 8], 4);
        const bool framed = magic == BATCH_MAGIC && off + 12 + (uint64_t)len <= log.size() &&
                            Crc32c(&log[off + 12], len) == crc;
        std::vector<KVBatch::Op> ops;
        bool ok = framed;
        if (framed) {
            const unsigned char* p = &log[off + 12];
            const unsigned char* end = p + len;
            while (ok && p < end) {
                const uint8_t op = *p++;
                uint64_t klen, vlen = 0;
                if (!GetVar(p, end, klen) || (uint64_t)(end - p) < klen) {
                    ok = false;
                    break;
                }
                std::string key((const char*)p, klen);
                p += klen;
                if (op == OP_PUT) {
                    if (!GetVar(p, end, vlen) || (uint64_t)(end - p) < vlen) {
                        ok = false;
                        break;
                    }
                    ops.push_back({true, std::move(key), std::string((const char*)p, vlen)});
                    p += vlen;
                } else if (op == OP_DEL) {
                    ops.push_back({false, std::move(key), std::string()});
                } else {
                    ok = false;
                }
            }
        }
        if (ok) { // apply the whole batch in log order
            for (auto& o : ops) {
                if (o.put)
                    out[o.key] = std::move(o.value);
                else
                    out.erase(o.key);
            }
            off += 12 + len;
            continue;
        }
        // damaged: resynchronise on the next batch header
        size_t next = off + 1;
        while (next + 4 <= log.size()) {
            uint32_t m;
            memcpy(&m, &log[next], 4);
            if (m == BATCH_MAGIC) break;
            ++next;
        }
        if (next + 4 > log.size()) next = log.size();
        if (skipped) *skipped += next - off;
        off = next;
    }
    if (skipped && off < log.size()) *skipped += log.size() - off;
    return out;
}

bool KVStore::WriteBatch(KVBatch& batch, bool fSync) {
    if (batch.ops.empty()) return true;
    std::lock_guard<std::mutex> l(cs);
    if (memOnly) {
        for (auto& op : batch.ops) {
            if (op.put) {
                auto it = index.find(op.key);
                if (it != index.end()) {
                    mem[it->second.off] = std::move(op.value);
                    it->second.len = (uint32_t)mem[it->second.off].size();
                } else {
                    mem.push_back(std::move(op.value));
                    index[op.key] = Loc{mem.size() - 1, (uint32_t)mem.back().size()};
                }
            } else {
                auto it = index.find(op.key);
                if (it != index.end()) {
                    mem[it->second.off].clear();
                    mem[it->second.off].shrink_to_fit();
                    index.erase(it);
                }
            }
        }
        batch.Clear();
        return true;
    }
    std::string payload;
    payload.reserve(batch.bytes + batch.ops.size() * 8);
    std::vector<std::pair<size_t, size_t>> valuePos; // payload offset of each put value
    for (const auto& op : batch.ops) {
        payload.push_back((char)(op.put ? OP_PUT : OP_DEL));
        PutVar(payload, op.key.size());
        payload += op.key;
        if (op.put) {
            PutVar(payload, op.value.size());
            valuePos.emplace_back(payload.size(), op.value.size());
            payload += op.value;
        } else {
            valuePos.emplace_back(0, 0);
        }
    }
    unsigned char hdr[12];
    const uint32_t magic = BATCH_MAGIC, len = (uint32_t)payload.size();
    const uint32_t crc = Crc32c((const unsigned char*)payload.data(), payload.size());
    memcpy(hdr, &magic, 4);
    memcpy(hdr + 4, &len, 4);
    memcpy(hdr + 8, &crc, 4);
    if (::lseek(fd, (off_t)logSize, SEEK_SET) < 0) return false;
    if (!WriteAll(fd, hdr, 12) || !WriteAll(fd, payload.data(), payload.size())) return false;
    if (fSync && ::fdatasync(fd) != 0) return false;
    const uint64_t base = logSize + 12;
    for (size_t i = 0; i < batch.ops.size(); i++) {
        const auto& op = batch.ops[i];
        auto it = index.find(op.key);
        if (it != index.end()) liveBytes -= it->second.len + it->first.size();
        if (op.put) {
            index[op.key] = Loc{base + valuePos[i].first, (uint32_t)valuePos[i].second};
            liveBytes += valuePos[i].second + op.key.size();
        } else if (it != index.end()) {
            index.erase(it);
        }
    }
    logSize += 12 + payload.size();
    batch.Clear();
    MaybeCompact();
    return true;
}

bool KVStore::ReadRaw(const std::string& key, std::string& value) const {
    std::lock_guard<std::mutex> l(cs);
    auto it = index.find(key);
    if (it == index.end()) return false;
    if (memOnly) {
        value = mem[it->second.off];
        return true;
    }
    value.resize(it->second.len);
    return it->second.len == 0 || PreadAll(fd, &value[0], it->second.len, it->second.off);
}

bool KVStore::ExistsRaw(const std::string& key) const {
    std::lock_guard<std::mutex> l(cs);
    return index.count(key) > 0;
}

bool KVStore::IsEmpty() const {
    std::lock_guard<std::mutex> l(cs);
    return index.empty();
}

size_t KVStore::Count() const {
    std::lock_guard<std::mutex> l(cs);
    return index.size();
}

size_t KVStore::EstimateSize(const std::string& begin, const std::string& end) const {
    std::lock_guard<std::mutex> l(cs);
    size_t n = 0;
    for (auto it = index.lower_bound(begin); it != index.end() && it->first < end; ++it)
        n += it->first.size() + it->second.len;
    return n;
}

void KVStore::MaybeCompact() {
    // called with cs held
    const uint64_t MIN_LOG = 64ull << 20;
    if (logSize > MIN_LOG && logSize > 3 * (liveBytes + index.size() * 8)) DoCompact();
}

void KVStore::DoCompact() {
    // called with cs held
    {
        std::string tmp = dir + "/kv.log.compact";
        int nfd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
        if (nfd < 0) return;
        uint64_t noff = 0;
        std::map<std::string, Loc> nindex;
        std::string payload, value;
        auto flush = [&](bool force) -> bool {
            if (payload.empty() || (!force && payload.size() < (4u << 20))) return true;
            unsigned char hdr[12];
            const uint32_t magic = BATCH_MAGIC, len = (uint32_t)payload.size();
            const uint32_t crc = Crc32c((const unsigned char*)payload.data(), payload.size());
            memcpy(hdr, &magic, 4);
            memcpy(hdr + 4, &len, 4);
            memcpy(hdr + 8, &crc, 4);
            if (!WriteAll(nfd, hdr, 12) || !WriteAll(nfd, payload.data(), payload.size())) return false;
            noff += 12 + payload.size();
            payload.clear();
            return true;
        };
        for (const auto& kv : index) {
            value.resize(kv.second.len);
            if (kv.second.len && !PreadAll(fd, &value[0], kv.second.len, kv.second.off)) {
                ::close(nfd);
                ::unlink(tmp.c_str());
                return;
            }
            payload.push_back((char)OP_PUT);
            PutVar(payload, kv.first.size());
            payload += kv.first;
            PutVar(payload, value.size());
            nindex[kv.first] = Loc{noff + 12 + payload.size(), kv.second.len};
            payload += value;
            if (payload.size() >= (4u << 20) && !flush(true)) {
                ::close(nfd);
                ::unlink(tmp.c_str());
                return;
            }
        }
        if (!flush(true) || ::fsync(nfd) != 0 || ::rename(tmp.c_str(), logPath.c_str()) != 0) {
            ::close(nfd);
            ::unlink(tmp.c_str());
            return;
        }
        ::close(fd);
        fd = nfd;
        index.swap(nindex);
        logSize = noff;
    }
}

void KVStore::Compact() {
    std::lock_guard<std::mutex> l(cs);
    if (!memOnly) DoCompact();
}

bool KVStore::NextKey(const std::string& from, bool inclusive, std::string& out) const {
    std::lock_guard<std::mutex> l(cs);
    auto it = inclusive ? index.lower_bound(from) : index.upper_bound(from);
    if (it == index.end()) return false;
    out = it->first;
    return true;
}

KVIterator::KVIterator(const KVStore* d) : db(d) {}
void KVIterator::Seek(const std::string& k) { valid = db->NextKey(k, true, curKey); }
void KVIterator::SeekToFirst() { valid = db->NextKey(std::string(), true, curKey); }
void KVIterator::Next() {
    if (valid) valid = db->NextKey(curKey, false, curKey);
}
bool KVIterator::RawValue(std::string& out) const { return valid && db->ReadRaw(curKey, out); }

} // namespace bcp
