#include "node/kvstore.h"

#include <algorithm>
#include <array>
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <fcntl.h>
#include <list>
#include <stdexcept>
#include <shared_mutex>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>
#include <unordered_map>

namespace bcp {

namespace {
const uint32_t BATCH_MAGIC_V1 = 0xB7C0DB01; // pre-segment records: payload = ops
const uint32_t BATCH_MAGIC = 0xB7C0DB02;    // payload = sequence number (8 bytes LE) + ops
const uint8_t OP_PUT = 1, OP_DEL = 2;
const uint64_t SEG_MAGIC = 0x3153474b56504342ull; // "BCPVKGS1"
const size_t FOOTER_BYTES = 64;

uint32_t Crc32cSoft(const unsigned char* p, size_t n) {
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
#if defined(__x86_64__)
// SSE4.2 crc32 instruction (same Castagnoli polynomial): ~10x the table loop on block reads
__attribute__((target("sse4.2"))) uint32_t Crc32cHw(const unsigned char* p, size_t n) {
    uint64_t c = 0xFFFFFFFFu;
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c = __builtin_ia32_crc32di(c, w);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = (uint32_t)c;
    while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
    return c32 ^ 0xFFFFFFFFu;
}
#endif
uint32_t Crc32c(const unsigned char* p, size_t n) {
#if defined(__x86_64__)
    static const bool hw = __builtin_cpu_supports("sse4.2");
    if (hw) return Crc32cHw(p, n);
#endif
    return Crc32cSoft(p, n);
}
uint32_t Crc32c(const std::string& s) { return Crc32c((const unsigned char*)s.data(), s.size()); }

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
void Put32(std::string& out, uint32_t v) { out.append((const char*)&v, 4); }
void Put64(std::string& out, uint64_t v) { out.append((const char*)&v, 8); }
uint32_t Get32(const unsigned char* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
uint64_t Get64(const unsigned char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
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
void SyncDir(const std::string& dir) {
    const int f = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (f >= 0) {
        ::fsync(f);
        ::close(f);
    }
}
uint64_t FileSize(const std::string& path) {
    struct stat st;
    return ::stat(path.c_str(), &st) == 0 ? (uint64_t)st.st_size : 0;
}
std::vector<std::string> ListDir(const std::string& dir) {
    std::vector<std::string> out;
    DIR* d = ::opendir(dir.c_str());
    if (!d) return out;
    while (dirent* e = ::readdir(d)) out.emplace_back(e->d_name);
    ::closedir(d);
    return out;
}
std::string Numbered(const std::string& dir, const char* prefix, uint64_t n, const char* ext) {
    char buf[64];
    snprintf(buf, sizeof(buf), "/%s-%06" PRIu64 ".%s", prefix, n, ext);
    return dir + buf;
}
// "<prefix>-<digits>.<ext>" -> n
bool ParseNumbered(const std::string& name, const std::string& prefix, const std::string& ext, uint64_t& n) {
    const std::string head = prefix + "-", tail = "." + ext;
    if (name.size() <= head.size() + tail.size() || name.compare(0, head.size(), head) != 0 ||
        name.compare(name.size() - tail.size(), tail.size(), tail) != 0)
        return false;
    const std::string digits = name.substr(head.size(), name.size() - head.size() - tail.size());
    if (digits.empty() || digits.size() > 18 || digits.find_first_not_of("0123456789") != std::string::npos) return false;
    n = std::stoull(digits);
    return true;
}

uint64_t Hash64(const char* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull; // FNV-1a, then a splitmix finaliser
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)p[i]) * 0x100000001b3ull;
    h ^= h >> 30;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 27;
    h *= 0x94d049bb133111ebull;
    return h ^ (h >> 31);
}

// position of a probe in an m-bit filter: multiply-shift range reduction instead of a division
inline uint64_t BloomBit(uint64_t x, uint64_t m) { return (uint64_t)(((unsigned __int128)x * m) >> 64); }

int CompareBytes(const char* a, size_t na, const char* b, size_t nb) {
    const int c = memcmp(a, b, std::min(na, nb));
    if (c) return c;
    return na < nb ? -1 : na > nb ? 1 : 0;
}

struct RecOp {
    bool put;
    std::string key, value;
};
bool DecodeOps(const unsigned char* p, const unsigned char* end, std::vector<RecOp>& ops) {
    while (p < end) {
        const uint8_t op = *p++;
        uint64_t klen, vlen = 0;
        if (!GetVar(p, end, klen) || (uint64_t)(end - p) < klen) return false;
        std::string key((const char*)p, klen);
        p += klen;
        if (op == OP_PUT) {
            if (!GetVar(p, end, vlen) || (uint64_t)(end - p) < vlen) return false;
            ops.push_back({true, std::move(key), std::string((const char*)p, vlen)});
            p += vlen;
        } else if (op == OP_DEL) {
            ops.push_back({false, std::move(key), std::string()});
        } else {
            return false;
        }
    }
    return true;
}

// Scan one log file: every well-framed batch record is handed to `apply` in order. Returns the
// offset just past the last good record (a torn / corrupt record ends the scan).
template <typename F> uint64_t ScanLog(int fd, uint64_t size, F&& apply) {
    uint64_t off = 0;
    std::vector<unsigned char> buf;
    while (off + 12 <= size) {
        unsigned char hdr[12];
        if (!PreadAll(fd, hdr, 12, off)) break;
        const uint32_t magic = Get32(hdr), len = Get32(hdr + 4), crc = Get32(hdr + 8);
        if ((magic != BATCH_MAGIC && magic != BATCH_MAGIC_V1) || off + 12 + len > size) break;
        buf.resize(len);
        if (len && !PreadAll(fd, buf.data(), len, off + 12)) break;
        if (Crc32c(buf.data(), len) != crc) break;
        const unsigned char* p = buf.data();
        uint64_t seq = 0;
        if (magic == BATCH_MAGIC) {
            if (len < 8) break;
            seq = Get64(p);
            p += 8;
        }
        std::vector<RecOp> ops;
        if (!DecodeOps(p, buf.data() + len, ops)) break;
        apply(magic == BATCH_MAGIC, seq, ops);
        off += 12 + len;
    }
    return off;
}

// ---------------------------------------------------------------- memtable
struct MemEntry {
    bool del = false;
    std::string value;
};
struct Memtable {
    std::map<std::string, MemEntry> m;
    size_t bytes = 0;
    static size_t Cost(size_t klen, size_t vlen) { return klen + vlen + 96; } // + node and string headers
    void Apply(RecOp& op, bool eraseDeletes) {
        auto it = m.find(op.key);
        if (it != m.end()) bytes -= Cost(it->first.size(), it->second.value.size());
        if (!op.put && eraseDeletes) {
            if (it != m.end()) m.erase(it);
            return;
        }
        if (it == m.end()) it = m.emplace(std::move(op.key), MemEntry()).first;
        it->second.del = !op.put;
        it->second.value = std::move(op.value);
        bytes += Cost(it->first.size(), it->second.value.size());
    }
};

// ---------------------------------------------------------------- block cache
class BlockCache {
public:
    explicit BlockCache(size_t cap) : cap(cap) {}
    std::shared_ptr<const std::string> Get(uint64_t key) {
        std::lock_guard<std::mutex> l(mu);
        auto it = map.find(key);
        if (it == map.end()) return nullptr;
        lru.splice(lru.begin(), lru, it->second);
        return it->second->second;
    }
    void Put(uint64_t key, std::shared_ptr<const std::string> v) {
        if (cap == 0) return;
        std::lock_guard<std::mutex> l(mu);
        if (map.count(key)) return;
        bytes += v->size() + 64;
        lru.emplace_front(key, std::move(v));
        map[key] = lru.begin();
        while (bytes > cap && !lru.empty()) {
            bytes -= lru.back().second->size() + 64;
            map.erase(lru.back().first);
            lru.pop_back();
        }
    }
    size_t Bytes() {
        std::lock_guard<std::mutex> l(mu);
        return bytes;
    }

private:
    std::mutex mu;
    size_t cap, bytes = 0;
    std::list<std::pair<uint64_t, std::shared_ptr<const std::string>>> lru;
    std::unordered_map<uint64_t, std::list<std::pair<uint64_t, std::shared_ptr<const std::string>>>::iterator> map;
};

struct Counters {
    std::atomic<uint64_t> flushes{0}, merges{0}, stalls{0}, bloomSkips{0}, blockReads{0};
};

// ---------------------------------------------------------------- segments
// File: data blocks (entries: varint klen, key, varint tag (0 = tombstone, else vlen + 1),
// value; then the block's CRC32C), the index (per block: varint klen, first key, varint offset,
// varint length incl. CRC; then CRC), the Bloom filter (k, bits; then CRC), a 64-byte footer
// (magic, index off/len, bloom off/len, keys, max batch sequence, CRC of those 56 bytes).
struct EntryView {
    const char* k;
    size_t klen;
    bool del;
    const char* v;
    size_t vlen;
};
bool NextEntry(const unsigned char*& p, const unsigned char* end, EntryView& e) {
    uint64_t klen, tag;
    if (!GetVar(p, end, klen) || (uint64_t)(end - p) < klen) return false;
    e.k = (const char*)p;
    e.klen = klen;
    p += klen;
    if (!GetVar(p, end, tag)) return false;
    e.del = tag == 0;
    e.vlen = tag ? tag - 1 : 0;
    if ((uint64_t)(end - p) < e.vlen) return false;
    e.v = (const char*)p;
    p += e.vlen;
    return true;
}

struct Segment {
    uint64_t id = 0;
    std::string path;
    int fd = -1;
    uint64_t fileBytes = 0, nkeys = 0, maxSeq = 0;
    std::string idxKeys;            // first keys of the blocks, concatenated
    std::vector<uint32_t> idxKeyOff; // nblocks + 1 offsets into idxKeys
    std::vector<uint64_t> blkOff;
    std::vector<uint32_t> blkLen; // incl. the CRC
    std::string bloom;
    int bloomK = 0;
    BlockCache* cache = nullptr;
    Counters* ctr = nullptr;
    std::atomic<bool> obsolete{false};

    ~Segment() {
        if (fd >= 0) ::close(fd);
        if (obsolete) ::unlink(path.c_str());
    }
    size_t NBlocks() const { return blkOff.size(); }
    int CompareFirst(size_t b, const std::string& key) const {
        return CompareBytes(idxKeys.data() + idxKeyOff[b], idxKeyOff[b + 1] - idxKeyOff[b], key.data(), key.size());
    }
    // last block whose first key <= key (-1: key sorts before the whole segment)
    long FindBlock(const std::string& key) const {
        long lo = 0, hi = (long)NBlocks() - 1, ans = -1;
        while (lo <= hi) {
            const long mid = (lo + hi) / 2;
            if (CompareFirst((size_t)mid, key) <= 0) {
                ans = mid;
                lo = mid + 1;
            } else {
                hi = mid - 1;
            }
        }
        return ans;
    }
    size_t IndexBytes() const { return idxKeys.size() + idxKeyOff.size() * 4 + blkOff.size() * 12; }
    bool MayContain(uint64_t h) const {
        if (bloomK == 0 || bloom.empty()) return true;
        const uint64_t m = (uint64_t)bloom.size() * 8;
        const uint64_t h2 = (h >> 33) | (h << 31);
        for (int i = 0; i < bloomK; i++) {
            const uint64_t bit = BloomBit(h + (uint64_t)i * h2, m);
            if (!((unsigned char)bloom[bit >> 3] & (1u << (bit & 7)))) return false;
        }
        return true;
    }
    // Block payload (CRC checked); `useCache` false for merges, which read every block once.
    std::shared_ptr<const std::string> Block(size_t b, bool useCache = true) const {
        const uint64_t ck = (id << 24) | (uint64_t)b;
        if (useCache && cache) {
            if (auto hit = cache->Get(ck)) return hit;
        }
        if (blkLen[b] < 4) return nullptr;
        std::string buf(blkLen[b], '\0');
        if (!PreadAll(fd, &buf[0], buf.size(), blkOff[b])) return nullptr;
        const uint32_t crc = Get32((const unsigned char*)buf.data() + buf.size() - 4);
        buf.resize(buf.size() - 4);
        if (Crc32c(buf) != crc) return nullptr;
        if (ctr) ctr->blockReads++;
        auto p = std::make_shared<const std::string>(std::move(buf));
        if (useCache && cache) cache->Put(ck, p);
        return p;
    }
    // 1: put (value set), 2: tombstone, 0: absent, -1: unreadable block
    int Get(const std::string& key, uint64_t h, std::string* value) const {
        if (!MayContain(h)) {
            if (ctr) ctr->bloomSkips++;
            return 0;
        }
        const long b = FindBlock(key);
        if (b < 0) return 0;
        auto blk = Block((size_t)b);
        if (!blk) return -1;
        const unsigned char* p = (const unsigned char*)blk->data();
        const unsigned char* end = p + blk->size();
        EntryView e;
        while (p < end) {
            if (!NextEntry(p, end, e)) return -1;
            const int c = CompareBytes(e.k, e.klen, key.data(), key.size());
            if (c == 0) {
                if (e.del) return 2;
                if (value) value->assign(e.v, e.vlen);
                return 1;
            }
            if (c > 0) return 0;
        }
        return 0;
    }

    static std::shared_ptr<Segment> Open(const std::string& path, uint64_t id, BlockCache* cache, Counters* ctr,
                                         std::string* err) {
        auto s = std::make_shared<Segment>();
        s->id = id;
        s->path = path;
        s->cache = cache;
        s->ctr = ctr;
        s->fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        auto fail = [&](const char* why) -> std::shared_ptr<Segment> {
            if (err) *err = path + ": " + why;
            return nullptr;
        };
        if (s->fd < 0) return fail("cannot open");
        struct stat st;
        if (fstat(s->fd, &st) != 0) return fail("cannot stat");
        s->fileBytes = (uint64_t)st.st_size;
        if (s->fileBytes < FOOTER_BYTES) return fail("too short");
        unsigned char f[FOOTER_BYTES];
        if (!PreadAll(s->fd, f, FOOTER_BYTES, s->fileBytes - FOOTER_BYTES)) return fail("footer unreadable");
        if (Get64(f) != SEG_MAGIC || Crc32c(f, 56) != Get32(f + 56)) return fail("bad footer");
        const uint64_t idxOff = Get64(f + 8), idxLen = Get64(f + 16), blOff = Get64(f + 24), blLen = Get64(f + 32);
        s->nkeys = Get64(f + 40);
        s->maxSeq = Get64(f + 48);
        if (idxLen < 4 || blLen < 5 || idxOff + idxLen > s->fileBytes || blOff + blLen > s->fileBytes)
            return fail("bad footer ranges");
        std::string idx(idxLen, '\0'), bl(blLen, '\0');
        if (!PreadAll(s->fd, &idx[0], idxLen, idxOff) || !PreadAll(s->fd, &bl[0], blLen, blOff))
            return fail("index unreadable");
        if (Crc32c((const unsigned char*)idx.data(), idxLen - 4) != Get32((const unsigned char*)idx.data() + idxLen - 4) ||
            Crc32c((const unsigned char*)bl.data(), blLen - 4) != Get32((const unsigned char*)bl.data() + blLen - 4))
            return fail("index or filter CRC");
        const unsigned char* p = (const unsigned char*)idx.data();
        const unsigned char* end = p + idxLen - 4;
        s->idxKeyOff.push_back(0);
        while (p < end) {
            uint64_t klen, off, len;
            if (!GetVar(p, end, klen) || (uint64_t)(end - p) < klen) return fail("index entry");
            s->idxKeys.append((const char*)p, klen);
            p += klen;
            if (!GetVar(p, end, off) || !GetVar(p, end, len) || off + len > idxOff) return fail("index entry");
            s->idxKeyOff.push_back((uint32_t)s->idxKeys.size());
            s->blkOff.push_back(off);
            s->blkLen.push_back((uint32_t)len);
        }
        s->idxKeys.shrink_to_fit();
        s->bloomK = (unsigned char)bl[0];
        s->bloom = bl.substr(1, blLen - 5);
        return s;
    }
};
typedef std::vector<std::shared_ptr<Segment>> SegList; // newest first

class SegmentWriter {
public:
    SegmentWriter(const std::string& path, const KVOptions& o, uint64_t expectedKeys) : path(path), opt(o) {
        const uint64_t bits = std::max<uint64_t>(64, expectedKeys * (uint64_t)std::max(1, opt.bloomBitsPerKey));
        bloom.assign((size_t)((bits + 7) / 8), '\0');
        k = std::max(1, std::min(30, (int)(opt.bloomBitsPerKey * 0.69)));
    }
    ~SegmentWriter() {
        if (fd >= 0) Abort();
    }
    bool Open() {
        fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
        return fd >= 0;
    }
    bool Add(const char* key, size_t klen, bool del, const char* value, size_t vlen) {
        if (block.empty()) firstKey.assign(key, klen);
        PutVar(block, klen);
        block.append(key, klen);
        PutVar(block, del ? 0 : vlen + 1);
        if (!del) block.append(value, vlen);
        const uint64_t h = Hash64(key, klen), h2 = (h >> 33) | (h << 31), m = (uint64_t)bloom.size() * 8;
        for (int i = 0; i < k; i++) {
            const uint64_t bit = BloomBit(h + (uint64_t)i * h2, m);
            bloom[bit >> 3] = (char)((unsigned char)bloom[bit >> 3] | (1u << (bit & 7)));
        }
        ++nkeys;
        return block.size() < opt.blockBytes || FlushBlock();
    }
    // Writes index, filter and footer, fsyncs and closes. False on any I/O error (file removed).
    bool Finish(uint64_t maxSeq) {
        if (!block.empty() && !FlushBlock()) return Abort();
        std::string idxTail = index;
        Put32(idxTail, Crc32c(index));
        std::string bl(1, (char)k);
        bl += bloom;
        Put32(bl, Crc32c(bl));
        const uint64_t idxOff = off, blOff = off + idxTail.size();
        std::string f;
        Put64(f, SEG_MAGIC);
        Put64(f, idxOff);
        Put64(f, idxTail.size());
        Put64(f, blOff);
        Put64(f, bl.size());
        Put64(f, nkeys);
        Put64(f, maxSeq);
        Put32(f, Crc32c(f));
        Put32(f, 0);
        if (!WriteAll(fd, idxTail.data(), idxTail.size()) || !WriteAll(fd, bl.data(), bl.size()) ||
            !WriteAll(fd, f.data(), f.size()) || ::fsync(fd) != 0)
            return Abort();
        ::close(fd);
        fd = -1;
        return true;
    }
    bool Abort() {
        if (fd >= 0) ::close(fd);
        fd = -1;
        ::unlink(path.c_str());
        return false;
    }
    uint64_t Keys() const { return nkeys; }

private:
    bool FlushBlock() {
        const uint32_t crc = Crc32c(block);
        Put32(block, crc);
        if (!WriteAll(fd, block.data(), block.size())) return false;
        PutVar(index, firstKey.size());
        index += firstKey;
        PutVar(index, off);
        PutVar(index, block.size());
        off += block.size();
        block.clear();
        return true;
    }
    std::string path;
    KVOptions opt;
    int fd = -1, k = 1;
    uint64_t off = 0, nkeys = 0;
    std::string block, firstKey, index, bloom;
};

// Forward cursor over one segment.
struct SegCursor {
    std::shared_ptr<Segment> seg;
    bool useCache = true;
    size_t b = 0;
    std::shared_ptr<const std::string> blk;
    const unsigned char *p = nullptr, *end = nullptr;
    bool valid = false, error = false;
    EntryView e{};

    void LoadBlock() {
        valid = false;
        while (b < seg->NBlocks()) {
            blk = seg->Block(b, useCache);
            if (!blk) {
                error = true;
                return;
            }
            p = (const unsigned char*)blk->data();
            end = p + blk->size();
            if (p < end) return;
            ++b;
        }
        blk.reset();
    }
    void Step() { // decode the next entry, crossing into later blocks
        for (;;) {
            if (blk && p < end) {
                if (!NextEntry(p, end, e)) {
                    error = true;
                    valid = false;
                    return;
                }
                valid = true;
                return;
            }
            if (blk) ++b;
            LoadBlock();
            if (!blk) {
                valid = false;
                return;
            }
        }
    }
    void SeekToFirst() {
        b = 0;
        blk.reset();
        LoadBlock();
        if (blk) Step();
    }
    void Seek(const std::string& target) {
        const long fb = seg->FindBlock(target);
        b = fb < 0 ? 0 : (size_t)fb;
        blk.reset();
        LoadBlock();
        if (!blk) return;
        Step();
        while (valid && CompareBytes(e.k, e.klen, target.data(), target.size()) < 0) Step();
    }
    int Cmp(const std::string& k) const { return CompareBytes(e.k, e.klen, k.data(), k.size()); }
};

} // namespace

// ---------------------------------------------------------------- store
struct KVStore::Impl {
    KVOptions opt;
    std::string dir;
    bool memOnly = false;

    mutable std::shared_mutex mu; // memtables, segment set, log, manifest (point reads share it)
    std::condition_variable_any cv;
    std::shared_ptr<Memtable> mem;
    std::shared_ptr<const Memtable> imm; // sealed, being written out
    uint64_t immSealLog = 0, immMaxSeq = 0;
    std::shared_ptr<const SegList> segs;
    int logFd = -1, lockFd = -1;
    uint64_t logNum = 0, logBytes = 0, firstLog = 0, nextFile = 1, seq = 0;
    bool stop = false, bgError = false, merging = false;
    std::atomic<bool> stopping{false}; // `stop` for loops that do not hold mu
    std::atomic<int> faults{0};        // KVStore::InjectFault bits (tests)

    std::mutex mergeMu; // one merge at a time (background merger or Compact())
    std::thread flusher, merger;
    BlockCache cache;
    Counters ctr;

    explicit Impl(const KVOptions& o) : opt(o), cache(o.blockCacheBytes) {}
    ~Impl() { Close(); } // also after a failed Open: threads joined, log and LOCK released

    std::string ManifestPath() const { return dir + "/MANIFEST"; }

    bool WriteManifestLocked() {
        if (faults.fetch_and(~KVStore::FAULT_MANIFEST) & KVStore::FAULT_MANIFEST) return false;
        std::string m = "BCPKV 1\n";
        m += "next " + std::to_string(nextFile) + "\n";
        m += "log " + std::to_string(firstLog) + "\n";
        m += "seq " + std::to_string(seq) + "\n";
        for (const auto& s : *segs) m += "seg " + std::to_string(s->id) + "\n";
        char crc[32];
        snprintf(crc, sizeof(crc), "crc %08x\n", Crc32c(m));
        m += crc;
        const std::string tmp = ManifestPath() + ".tmp";
        const int f = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
        if (f < 0) return false;
        const bool ok = WriteAll(f, m.data(), m.size()) && ::fsync(f) == 0;
        ::close(f);
        if (!ok || ::rename(tmp.c_str(), ManifestPath().c_str()) != 0) return false;
        SyncDir(dir);
        return true;
    }

    // -> false if absent; throws on a corrupt manifest
    bool ReadManifest(std::vector<uint64_t>& ids, uint64_t& next, uint64_t& log, uint64_t& sq) {
        const int f = ::open(ManifestPath().c_str(), O_RDONLY | O_CLOEXEC);
        if (f < 0) return false;
        std::string m(FileSize(ManifestPath()), '\0');
        const bool ok = m.empty() || PreadAll(f, &m[0], m.size(), 0);
        ::close(f);
        const size_t c = m.rfind("crc ");
        if (!ok || c == std::string::npos) throw std::runtime_error("KVStore: unreadable manifest in " + dir);
        const uint32_t want = (uint32_t)strtoul(m.c_str() + c + 4, nullptr, 16);
        if (Crc32c((const unsigned char*)m.data(), c) != want) throw std::runtime_error("KVStore: corrupt manifest in " + dir);
        size_t pos = 0;
        while (pos < c) {
            const size_t eol = m.find('\n', pos);
            const std::string line = m.substr(pos, eol - pos);
            pos = eol + 1;
            const size_t sp = line.find(' ');
            const std::string k = line.substr(0, sp), v = sp == std::string::npos ? "" : line.substr(sp + 1);
            if (k == "next") next = std::stoull(v);
            else if (k == "log") log = std::stoull(v);
            else if (k == "seq") sq = std::stoull(v);
            else if (k == "seg") ids.push_back(std::stoull(v));
        }
        return true;
    }

    bool OpenLog(uint64_t n, bool truncateTo, uint64_t size) {
        const std::string p = Numbered(dir, "kv", n, "log");
        const int f = ::open(p.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0600);
        if (f < 0) return false;
        if (truncateTo && ::ftruncate(f, (off_t)size) != 0) {
            ::close(f);
            return false;
        }
        if (::lseek(f, (off_t)size, SEEK_SET) < 0) {
            ::close(f);
            return false;
        }
        if (logFd >= 0) ::close(logFd);
        logFd = f;
        logNum = n;
        logBytes = size;
        return true;
    }

    void Open(const std::string& path, bool wipe) {
        dir = path;
        mem = std::make_shared<Memtable>();
        segs = std::make_shared<const SegList>();
        if (memOnly) return;
        MkdirP(dir);
        // one instance per directory (two would interleave logs and manifests)
        lockFd = ::open((dir + "/LOCK").c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
        if (lockFd < 0 || ::flock(lockFd, LOCK_EX | LOCK_NB) != 0)
            throw std::runtime_error("KVStore: " + dir + " is in use by another instance");
        const std::vector<std::string> names = ListDir(dir);
        if (wipe) {
            for (const std::string& n : names) {
                uint64_t x;
                if (n == "MANIFEST" || n == "MANIFEST.tmp" || n == "kv.log" || ParseNumbered(n, "kv", "log", x) ||
                    ParseNumbered(n, "seg", "sst", x) || (n.size() > 4 && n.compare(n.size() - 4, 4, ".tmp") == 0))
                    ::unlink((dir + "/" + n).c_str());
            }
        }
        std::vector<uint64_t> ids;
        uint64_t mnext = 1, mlog = 0;
        const bool haveManifest = !wipe && ReadManifest(ids, mnext, mlog, seq);
        SegList list;
        for (uint64_t id : ids) {
            std::string err;
            auto s = Segment::Open(Numbered(dir, "seg", id, "sst"), id, &cache, &ctr, &err);
            if (!s) throw std::runtime_error("KVStore: " + err);
            list.push_back(s);
        }
        segs = std::make_shared<const SegList>(std::move(list));
        // numbering, orphans (segments a crashed flush/merge left behind, logs already flushed)
        uint64_t maxSeen = 0;
        std::vector<uint64_t> logs;
        for (const std::string& n : wipe ? std::vector<std::string>() : ListDir(dir)) {
            uint64_t x;
            if (ParseNumbered(n, "seg", "sst", x)) {
                maxSeen = std::max(maxSeen, x);
                if (std::find(ids.begin(), ids.end(), x) == ids.end()) ::unlink((dir + "/" + n).c_str());
            } else if (ParseNumbered(n, "kv", "log", x)) {
                maxSeen = std::max(maxSeen, x);
                if (haveManifest && x < mlog) ::unlink((dir + "/" + n).c_str());
                else logs.push_back(x);
            } else if (n == "MANIFEST.tmp") {
                ::unlink((dir + "/" + n).c_str());
            }
        }
        nextFile = std::max(mnext, maxSeen + 1);
        std::sort(logs.begin(), logs.end());
        // a pre-segment store: replay its single log, then migrate it into a segment below
        // (with a manifest present it was migrated already and only its unlink was lost)
        const std::string legacy = dir + "/kv.log";
        const bool migrate = !wipe && !haveManifest && FileSize(legacy) > 0;
        if (haveManifest) ::unlink(legacy.c_str());
        auto replay = [&](const std::string& p, bool truncate) -> uint64_t {
            const int f = ::open(p.c_str(), O_RDWR | O_CLOEXEC);
            if (f < 0) return 0;
            const uint64_t size = FileSize(p);
            const uint64_t good = ScanLog(f, size, [&](bool v2, uint64_t s, std::vector<RecOp>& ops) {
                seq = v2 ? std::max(seq, s) : seq + 1;
                for (auto& op : ops) mem->Apply(op, false);
            });
            if (truncate && good != size && ::ftruncate(f, (off_t)good) != 0)
                throw std::runtime_error("KVStore: cannot truncate " + p);
            ::close(f);
            return good;
        };
        if (migrate) replay(legacy, false);
        uint64_t lastSize = 0;
        for (uint64_t n : logs) lastSize = replay(Numbered(dir, "kv", n, "log"), true);
        // keep appending to the newest log; the first log still needed stays as the manifest said
        bool ok;
        if (!logs.empty()) {
            firstLog = haveManifest ? std::max(mlog, logs.front()) : logs.front();
            ok = OpenLog(logs.back(), false, lastSize);
        } else {
            firstLog = nextFile++;
            ok = OpenLog(firstLog, true, 0);
        }
        if (!ok) throw std::runtime_error("KVStore: cannot open the log in " + dir);
        if (!migrate) { // a migration's first manifest is the flush's: until then kv.log stays authoritative
            std::lock_guard<std::shared_mutex> l(mu);
            if (!WriteManifestLocked()) throw std::runtime_error("KVStore: cannot write the manifest in " + dir);
        }
        flusher = std::thread([this] { FlusherLoop(); });
        merger = std::thread([this] { MergerLoop(); });
        if (migrate) {
            FlushAndWait();
            std::lock_guard<std::shared_mutex> l(mu);
            if (bgError || segs->empty()) throw std::runtime_error("KVStore: migrating " + legacy + " failed");
            ::unlink(legacy.c_str());
            SyncDir(dir);
        }
    }

    void Close() {
        {
            std::lock_guard<std::shared_mutex> l(mu);
            stop = true;
            stopping = true;
        }
        cv.notify_all();
        if (flusher.joinable()) flusher.join();
        if (merger.joinable()) merger.join();
        if (logFd >= 0) {
            ::fdatasync(logFd);
            ::close(logFd);
            logFd = -1;
        }
        if (lockFd >= 0) {
            ::close(lockFd); // releases the flock
            lockFd = -1;
        }
    }

    bool NeedFlushLocked() const {
        if (mem->m.empty()) return false;
        const size_t logCap = std::max<size_t>(2 * opt.memtableBytes, 1u << 20);
        return mem->bytes >= opt.memtableBytes || logBytes >= logCap;
    }

    // Seal the memtable: a fresh log takes the next writes; the flusher writes `imm` out.
    bool SealLocked(std::unique_lock<std::shared_mutex>& l) {
        // back-pressure: a second full memtable, or merges far behind (reads would check too
        // many segments), waits for the background threads
        while ((imm || (int)segs->size() > 3 * opt.maxSegments) && !bgError && !stop) {
            ctr.stalls++;
            cv.wait(l);
        }
        if (bgError) return false;
        const uint64_t n = nextFile++;
        if (::fdatasync(logFd) != 0 || !OpenLog(n, true, 0)) {
            bgError = true;
            return false;
        }
        imm = mem;
        immSealLog = n;
        immMaxSeq = seq;
        mem = std::make_shared<Memtable>();
        cv.notify_all();
        return true;
    }

    std::shared_ptr<Segment> WriteSegment(const Memtable& m, uint64_t maxSeq) {
        if (faults.fetch_and(~KVStore::FAULT_SEGMENT) & KVStore::FAULT_SEGMENT) return nullptr;
        uint64_t id;
        {
            std::lock_guard<std::shared_mutex> l(mu);
            id = nextFile++;
        }
        const std::string path = Numbered(dir, "seg", id, "sst");
        SegmentWriter w(path, opt, m.m.size());
        if (!w.Open()) return nullptr;
        for (const auto& kv : m.m)
            if (!w.Add(kv.first.data(), kv.first.size(), kv.second.del, kv.second.value.data(), kv.second.value.size()))
                return nullptr;
        if (!w.Finish(maxSeq)) return nullptr;
        return Segment::Open(path, id, &cache, &ctr, nullptr);
    }

    void FlusherLoop() {
        std::unique_lock<std::shared_mutex> l(mu);
        for (;;) {
            cv.wait(l, [&] { return stop || imm; });
            if (!imm) return; // stop, nothing pending
            auto m = imm;
            const uint64_t sealLog = immSealLog, maxSeq = immMaxSeq;
            l.unlock();
            auto seg = WriteSegment(*m, maxSeq);
            l.lock();
            if (!seg) {
                // the sealed memtable stays readable (its keys are in no segment) and its logs
                // stay on disk for the replay at the next open; no further writes are taken
                bgError = true;
                cv.notify_all();
                return;
            }
            auto next = std::make_shared<SegList>(*segs);
            next->insert(next->begin(), seg);
            segs = next;
            const uint64_t oldFirst = firstLog;
            firstLog = sealLog;
            imm.reset();
            ctr.flushes++;
            if (!WriteManifestLocked()) {
                // the manifest on disk still names the previous segments and the previous first
                // log: keep those logs for the replay (the new segment, unnamed there, serves the
                // keys until then and is discarded at the next open)
                bgError = true;
                cv.notify_all();
                return;
            }
            for (uint64_t n = oldFirst; n < sealLog; n++) ::unlink(Numbered(dir, "kv", n, "log").c_str());
            cv.notify_all();
        }
    }

    bool NeedMergeLocked() const { return !merging && (int)segs->size() > opt.maxSegments; }

    void MergerLoop() {
        std::unique_lock<std::shared_mutex> l(mu);
        for (;;) {
            cv.wait(l, [&] { return stop || NeedMergeLocked(); });
            if (stop) return;
            l.unlock();
            Merge(false);
            l.lock();
        }
    }

    // Merge a run of adjacent segments (all of them when `full`) into one.
    bool Merge(bool full) {
        std::lock_guard<std::mutex> mg(mergeMu);
        std::shared_ptr<const SegList> cur;
        {
            std::lock_guard<std::shared_mutex> l(mu);
            cur = segs;
            if (cur->empty() || (!full && (int)cur->size() <= opt.maxSegments)) return true;
            merging = true;
        }
        size_t lo = 0, hi = cur->size();
        if (!full) { // the window of mergeWidth adjacent segments with the fewest bytes
            const size_t w = std::min(cur->size(), (size_t)std::max(2, opt.mergeWidth));
            uint64_t best = UINT64_MAX;
            for (size_t i = 0; i + w <= cur->size(); i++) {
                uint64_t t = 0;
                for (size_t j = i; j < i + w; j++) t += (*cur)[j]->fileBytes;
                if (t < best) {
                    best = t;
                    lo = i;
                }
            }
            hi = lo + w;
        }
        const bool dropTombstones = hi == cur->size();
        uint64_t expected = 0, maxSeq = 0;
        std::vector<SegCursor> cs(hi - lo);
        for (size_t i = lo; i < hi; i++) {
            cs[i - lo].seg = (*cur)[i];
            cs[i - lo].useCache = false;
            cs[i - lo].SeekToFirst();
            expected += (*cur)[i]->nkeys;
            maxSeq = std::max(maxSeq, (*cur)[i]->maxSeq);
        }
        uint64_t id;
        {
            std::lock_guard<std::shared_mutex> l(mu);
            id = nextFile++;
        }
        const std::string path = Numbered(dir, "seg", id, "sst");
        auto done = [&](bool ok) {
            std::lock_guard<std::shared_mutex> l(mu);
            merging = false;
            if (!ok) bgError = true;
            cv.notify_all();
            return ok;
        };
        SegmentWriter w(path, opt, expected);
        if (!w.Open()) return done(false);
        std::string last;
        for (;;) {
            int win = -1;
            for (size_t i = 0; i < cs.size(); i++) {
                if (cs[i].error) return done(false);
                if (!cs[i].valid) continue;
                if (win < 0 || CompareBytes(cs[i].e.k, cs[i].e.klen, cs[win].e.k, cs[win].e.klen) < 0) win = (int)i;
            }
            if (win < 0) break;
            if (stopping.load(std::memory_order_relaxed)) { // (no lock per entry: writers hold mu for whole batches)
                w.Abort();
                std::lock_guard<std::shared_mutex> l(mu);
                merging = false;
                return false;
            }
            const EntryView e = cs[win].e; // newest copy (lowest index) wins ties
            last.assign(e.k, e.klen);
            if (!(e.del && dropTombstones) && !w.Add(e.k, e.klen, e.del, e.v, e.vlen)) return done(false);
            for (auto& c : cs)
                while (c.valid && c.Cmp(last) == 0) c.Step();
        }
        std::shared_ptr<Segment> seg;
        const bool empty = w.Keys() == 0;
        if (!w.Finish(maxSeq)) return done(false);
        if (!empty) {
            seg = Segment::Open(path, id, &cache, &ctr, nullptr);
            if (!seg) return done(false);
        } else {
            ::unlink(path.c_str());
        }
        {
            std::lock_guard<std::shared_mutex> l(mu);
            // flushes only add at the front: the window is still contiguous, shifted
            auto next = std::make_shared<SegList>(*segs);
            auto it = std::find(next->begin(), next->end(), (*cur)[lo]);
            if (it == next->end() || (size_t)(next->end() - it) < hi - lo) {
                merging = false;
                bgError = true;
                cv.notify_all();
                return false;
            }
            it = next->erase(it, it + (hi - lo));
            if (seg) next->insert(it, seg);
            const auto before = segs;
            segs = next;
            if (!WriteManifestLocked()) {
                // the manifest on disk still names the inputs: keep serving (and keeping) them,
                // and drop the merged segment the manifest does not know
                segs = before;
                if (seg) seg->obsolete = true;
                merging = false;
                bgError = true;
                cv.notify_all();
                return false;
            }
            for (size_t i = lo; i < hi; i++) (*cur)[i]->obsolete = true; // unlinked when released
            ctr.merges++;
            merging = false;
            cv.notify_all();
        }
        return true;
    }

    void FlushAndWait() {
        std::unique_lock<std::shared_mutex> l(mu);
        if (memOnly) return;
        if (!mem->m.empty() && !SealLocked(l)) return;
        cv.wait(l, [&] { return !imm || bgError; }); // also a memtable sealed by an earlier write
    }
};

KVStore::KVStore(const std::string& path, bool memory_only, bool wipe, const KVOptions& opts)
    : d(new Impl(opts)) {
    d->memOnly = memory_only;
    d->Open(path, wipe);
}

KVStore::~KVStore() {}

void KVStore::InjectFault(int what) { d->faults.fetch_or(what); }

bool KVStore::WriteBatch(KVBatch& batch, bool fSync) {
    if (batch.ops.empty()) return true;
    std::unique_lock<std::shared_mutex> l(d->mu);
    if (d->bgError) return false;
    const uint64_t seq = ++d->seq;
    std::vector<RecOp> ops;
    ops.reserve(batch.ops.size());
    if (!d->memOnly) {
        std::string payload;
        payload.reserve(8 + batch.bytes + batch.ops.size() * 8);
        Put64(payload, seq);
        for (const auto& op : batch.ops) {
            payload.push_back((char)(op.put ? OP_PUT : OP_DEL));
            PutVar(payload, op.key.size());
            payload += op.key;
            if (op.put) {
                PutVar(payload, op.value.size());
                payload += op.value;
            }
        }
        std::string hdr;
        Put32(hdr, BATCH_MAGIC);
        Put32(hdr, (uint32_t)payload.size());
        Put32(hdr, Crc32c(payload));
        if (!WriteAll(d->logFd, hdr.data(), hdr.size()) || !WriteAll(d->logFd, payload.data(), payload.size())) {
            // a partial record would be dropped on replay; refuse further writes to keep order
            d->bgError = true;
            return false;
        }
        d->logBytes += hdr.size() + payload.size();
        if (fSync && ::fdatasync(d->logFd) != 0) return false;
    }
    for (auto& op : batch.ops) {
        RecOp r{op.put, std::move(op.key), std::move(op.value)};
        d->mem->Apply(r, d->memOnly);
    }
    batch.Clear();
    if (!d->memOnly && d->NeedFlushLocked()) d->SealLocked(l); // a failure surfaces on the next write
    return true;
}

bool KVStore::ReadRaw(const std::string& key, std::string& value) const {
    std::shared_ptr<const SegList> s;
    {
        std::shared_lock<std::shared_mutex> l(d->mu);
        auto it = d->mem->m.find(key);
        if (it != d->mem->m.end()) {
            if (it->second.del) return false;
            value = it->second.value;
            return true;
        }
        if (d->imm) {
            auto jt = d->imm->m.find(key);
            if (jt != d->imm->m.end()) {
                if (jt->second.del) return false;
                value = jt->second.value;
                return true;
            }
        }
        s = d->segs;
    }
    if (s->empty()) return false;
    const uint64_t h = Hash64(key.data(), key.size());
    for (const auto& seg : *s) {
        const int r = seg->Get(key, h, &value);
        if (r == 1) return true;
        if (r == 2) return false; // tombstone
        if (r < 0) throw KVCorruption("KVStore: unreadable block in " + seg->path);
    }
    return false;
}

void KVStore::ReadRawMany(const std::string* keys, size_t n, std::string* values, uint8_t* found) const {
    std::shared_ptr<const SegList> s;
    std::vector<size_t> rest; // not decided by the memtables
    {
        std::shared_lock<std::shared_mutex> l(d->mu);
        for (size_t i = 0; i < n; i++) {
            found[i] = 0;
            auto it = d->mem->m.find(keys[i]);
            if (it != d->mem->m.end()) {
                if (!it->second.del) {
                    values[i] = it->second.value;
                    found[i] = 1;
                }
                continue;
            }
            if (d->imm) {
                auto jt = d->imm->m.find(keys[i]);
                if (jt != d->imm->m.end()) {
                    if (!jt->second.del) {
                        values[i] = jt->second.value;
                        found[i] = 1;
                    }
                    continue;
                }
            }
            rest.push_back(i);
        }
        s = d->segs;
    }
    if (s->empty()) return;
    for (size_t i : rest) {
        const uint64_t h = Hash64(keys[i].data(), keys[i].size());
        for (const auto& seg : *s) {
            const int r = seg->Get(keys[i], h, &values[i]);
            if (r < 0) throw KVCorruption("KVStore: unreadable block in " + seg->path);
            if (r == 1) found[i] = 1;
            if (r != 0) break; // found, or a tombstone
        }
    }
}

bool KVStore::ExistsRaw(const std::string& key) const {
    std::string v;
    return ReadRaw(key, v);
}

bool KVStore::IsEmpty() const {
    KVIterator it(this);
    it.SeekToFirst();
    return !it.Valid();
}

size_t KVStore::Count() const {
    size_t n = 0;
    KVIterator it(this);
    for (it.SeekToFirst(); it.Valid(); it.Next()) ++n;
    return n;
}

size_t KVStore::EstimateSize(const std::string& begin, const std::string& end) const {
    std::shared_ptr<const SegList> s;
    size_t n = 0;
    {
        std::lock_guard<std::shared_mutex> l(d->mu);
        for (auto* m : {d->mem.get(), const_cast<Memtable*>(d->imm.get())}) {
            if (!m) continue;
            for (auto it = m->m.lower_bound(begin); it != m->m.end() && it->first < end; ++it)
                n += it->first.size() + it->second.value.size();
        }
        s = d->segs;
    }
    for (const auto& seg : *s) {
        if (seg->NBlocks() == 0) continue;
        const long b0 = std::max(0L, seg->FindBlock(begin)), b1 = seg->FindBlock(end);
        for (long b = b0; b <= b1 && b < (long)seg->NBlocks(); b++) n += seg->blkLen[(size_t)b];
    }
    return n;
}

void KVStore::Flush() { d->FlushAndWait(); }

void KVStore::Compact() {
    if (d->memOnly) return;
    d->FlushAndWait();
    d->Merge(true);
}

uint64_t KVStore::LogBytes() const {
    std::lock_guard<std::shared_mutex> l(d->mu);
    uint64_t n = d->logBytes;
    for (const auto& s : *d->segs) n += s->fileBytes;
    return n;
}

KVStats KVStore::Stats() const {
    KVStats st;
    std::lock_guard<std::shared_mutex> l(d->mu);
    st.segments = d->segs->size();
    for (const auto& s : *d->segs) {
        st.segmentBytes += s->fileBytes;
        st.indexBytes += s->IndexBytes();
        st.bloomBytes += s->bloom.size();
    }
    st.logBytes = d->logBytes;
    st.memtableBytes = d->mem->bytes;
    st.immutableBytes = d->imm ? d->imm->bytes : 0;
    st.cacheBytes = d->cache.Bytes();
    st.flushes = d->ctr.flushes;
    st.merges = d->ctr.merges;
    st.stalls = d->ctr.stalls;
    st.bloomSkips = d->ctr.bloomSkips;
    st.blockReads = d->ctr.blockReads;
    return st;
}

std::map<std::string, std::string> KVStore::Salvage(const std::string& dir, uint64_t* skipped) {
    std::map<std::string, std::string> out;
    uint64_t skip = 0;
    const std::vector<std::string> names = ListDir(dir);
    // segments, oldest data first (their footers carry the last batch they contain)
    std::vector<std::shared_ptr<Segment>> segs;
    std::vector<uint64_t> logs;
    for (const std::string& n : names) {
        uint64_t x;
        if (ParseNumbered(n, "seg", "sst", x)) {
            auto s = Segment::Open(dir + "/" + n, x, nullptr, nullptr, nullptr);
            if (s) segs.push_back(s);
            else skip += FileSize(dir + "/" + n);
        } else if (ParseNumbered(n, "kv", "log", x)) {
            logs.push_back(x);
        }
    }
    std::sort(segs.begin(), segs.end(), [](const std::shared_ptr<Segment>& a, const std::shared_ptr<Segment>& b) {
        return a->maxSeq != b->maxSeq ? a->maxSeq < b->maxSeq : a->id < b->id;
    });
    uint64_t segSeq = 0;
    for (const auto& s : segs) {
        segSeq = std::max(segSeq, s->maxSeq);
        for (size_t b = 0; b < s->NBlocks(); b++) {
            auto blk = s->Block(b, false);
            if (!blk) {
                skip += s->blkLen[b];
                continue;
            }
            const unsigned char* p = (const unsigned char*)blk->data();
            const unsigned char* end = p + blk->size();
            EntryView e;
            while (p < end && NextEntry(p, end, e)) {
                if (e.del) out.erase(std::string(e.k, e.klen));
                else out[std::string(e.k, e.klen)] = std::string(e.v, e.vlen);
            }
        }
    }
    // logs: the pre-segment kv.log, then kv-<n>.log in order; batches a segment already holds
    // are skipped, damaged stretches resynchronised on the next record header
    std::sort(logs.begin(), logs.end());
    std::vector<std::string> paths;
    if (FileSize(dir + "/kv.log") > 0) paths.push_back(dir + "/kv.log");
    for (uint64_t n : logs) paths.push_back(Numbered(dir, "kv", n, "log"));
    for (const std::string& path : paths) {
        const int f = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        if (f < 0) continue;
        std::vector<unsigned char> log(FileSize(path));
        const bool ok = log.empty() || PreadAll(f, log.data(), log.size(), 0);
        ::close(f);
        if (!ok) continue;
        size_t off = 0;
        while (off + 12 <= log.size()) {
            const uint32_t magic = Get32(&log[off]), len = Get32(&log[off + 4]), crc = Get32(&log[off + 8]);
            const bool framed = (magic == BATCH_MAGIC || magic == BATCH_MAGIC_V1) && off + 12 + (uint64_t)len <= log.size() &&
                                Crc32c(&log[off + 12], len) == crc && (magic == BATCH_MAGIC_V1 || len >= 8);
            std::vector<RecOp> ops;
            bool good = framed;
            uint64_t seq = 0;
            if (framed) {
                const unsigned char* p = &log[off + 12];
                if (magic == BATCH_MAGIC) {
                    seq = Get64(p);
                    p += 8;
                }
                good = DecodeOps(p, &log[off + 12] + len, ops);
            }
            if (good) {
                if (magic == BATCH_MAGIC_V1 || seq > segSeq) {
                    for (auto& o : ops) {
                        if (o.put) out[o.key] = std::move(o.value);
                        else out.erase(o.key);
                    }
                }
                off += 12 + len;
                continue;
            }
            size_t next = off + 1;
            while (next + 4 <= log.size()) {
                const uint32_t m = Get32(&log[next]);
                if (m == BATCH_MAGIC || m == BATCH_MAGIC_V1) break;
                ++next;
            }
            if (next + 4 > log.size()) next = log.size();
            skip += next - off;
            off = next;
        }
        if (off < log.size()) skip += log.size() - off;
    }
    if (skipped) *skipped = skip;
    return out;
}

// ---------------------------------------------------------------- iterator
struct KVIterator::State {
    std::shared_ptr<const Memtable> imm;
    std::map<std::string, MemEntry>::const_iterator immIt;
    std::shared_ptr<const SegList> segs;
    std::vector<SegCursor> cur;
    bool memValid = false;
    std::string memKey;
    MemEntry memEnt;
};

KVIterator::KVIterator(const KVStore* d) : db(d), st(new State) {}
KVIterator::~KVIterator() {}

void KVIterator::Seek(const std::string& k) {
    KVStore::Impl& I = *db->d;
    {
        std::lock_guard<std::shared_mutex> l(I.mu);
        st->imm = I.imm;
        st->segs = I.segs;
        auto it = I.mem->m.lower_bound(k);
        st->memValid = it != I.mem->m.end();
        if (st->memValid) {
            st->memKey = it->first;
            st->memEnt = it->second;
        }
    }
    if (st->imm) st->immIt = st->imm->m.lower_bound(k);
    st->cur.assign(st->segs->size(), SegCursor());
    for (size_t i = 0; i < st->segs->size(); i++) {
        st->cur[i].seg = (*st->segs)[i];
        st->cur[i].Seek(k);
    }
    Settle();
}

void KVIterator::SeekToFirst() { Seek(std::string()); }

void KVIterator::Next() {
    if (valid) Settle();
}

void KVIterator::Settle() {
    KVStore::Impl& I = *db->d;
    State& s = *st;
    for (;;) {
        // smallest current key; on ties the newest source wins (memtable, sealed memtable, segments)
        int src = -2; // -1 memtable, -2 none, 0.. = imm (0) then segment i + 1
        const char* bk = nullptr;
        size_t bl = 0;
        auto consider = [&](int id, const char* k, size_t kl) {
            if (src == -2 || CompareBytes(k, kl, bk, bl) < 0) {
                src = id;
                bk = k;
                bl = kl;
            }
        };
        if (s.memValid) consider(-1, s.memKey.data(), s.memKey.size());
        if (s.imm && s.immIt != s.imm->m.end()) consider(0, s.immIt->first.data(), s.immIt->first.size());
        for (size_t i = 0; i < s.cur.size(); i++)
            if (s.cur[i].valid) consider((int)i + 1, s.cur[i].e.k, s.cur[i].e.klen);
        if (src == -2) {
            valid = false;
            return;
        }
        std::string key(bk, bl);
        bool del;
        std::string value;
        if (src == -1) {
            del = s.memEnt.del;
            value = s.memEnt.value;
        } else if (src == 0) {
            del = s.immIt->second.del;
            value = s.immIt->second.value;
        } else {
            const EntryView& e = s.cur[(size_t)src - 1].e;
            del = e.del;
            value.assign(e.v, e.vlen);
        }
        // advance every source past `key`
        {
            std::lock_guard<std::shared_mutex> l(I.mu);
            auto it = I.mem->m.upper_bound(key);
            s.memValid = it != I.mem->m.end();
            if (s.memValid) {
                s.memKey = it->first;
                s.memEnt = it->second;
            }
        }
        if (s.imm)
            while (s.immIt != s.imm->m.end() && s.immIt->first <= key) ++s.immIt;
        for (auto& c : s.cur)
            while (c.valid && c.Cmp(key) <= 0) c.Step();
        if (del) continue;
        curKey = std::move(key);
        curValue = std::move(value);
        valid = true;
        return;
    }
}

} // namespace bcp
