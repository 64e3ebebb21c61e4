#include "wallet/bdbimport.h"
#include "util/lockedpool.h"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <set>
#include <sys/stat.h>

namespace bcp {

namespace {

// On-disk layout (Berkeley DB 4.x db_page.h; all integers in the file's byte order, little-endian here).
constexpr uint32_t BTREE_MAGIC = 0x053162;
constexpr size_t META_MAGIC = 12, META_PAGESIZE = 20, META_TYPE = 25, META_METAFLAGS = 26, META_LASTPG = 32,
                 META_FLAGS = 48, META_ROOT = 88;
constexpr uint32_t BTM_SUBDB = 0x20;      // DBMETA.flags: the file's master database lists sub-databases
constexpr uint8_t DBMETA_CHKSUM = 0x01;   // DBMETA.metaflags: pages carry checksums
constexpr size_t PAGE_NEXT = 16, PAGE_ENTRIES = 20, PAGE_HFOFF = 22, PAGE_TYPE = 25, PAGE_HDR = 26;
constexpr uint8_t P_IBTREE = 3, P_LBTREE = 5, P_OVERFLOW = 7, P_BTREEMETA = 9;
constexpr uint8_t B_KEYDATA = 1, B_OVERFLOW = 3, B_DELETE = 0x80;

uint16_t U16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t U32(const unsigned char* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

class BtreeFile {
public:
    explicit BtreeFile(std::string bytes) : f(std::move(bytes)) {}
    ~BtreeFile() { memory_cleanse(&f[0], f.size()); } // the file holds plaintext key records

    bool Open(std::string& err) {
        if (f.size() < 512) return Fail(err, "file too short for a database");
        const unsigned char* m = P0();
        const uint32_t magic = U32(m + META_MAGIC);
        if (magic != BTREE_MAGIC) {
            if (magic == 0x62310500) return Fail(err, "big-endian Berkeley DB file (not supported)");
            return Fail(err, "not a Berkeley DB btree file");
        }
        if (m[META_TYPE] != P_BTREEMETA) return Fail(err, "unexpected meta page type");
        if (m[META_METAFLAGS] & DBMETA_CHKSUM) return Fail(err, "checksummed or encrypted pages (not supported)");
        pagesize = U32(m + META_PAGESIZE);
        if (pagesize < 512 || pagesize > 65536 || (pagesize & (pagesize - 1))) return Fail(err, "bad page size");
        npages = f.size() / pagesize;
        if (U32(m + META_LASTPG) >= npages) return Fail(err, "truncated file (last page beyond the end)");
        return true;
    }

    // records of the tree whose meta page is `metaPg`
    bool Records(uint32_t metaPg, BdbRecords& out, std::string& err) {
        const unsigned char* meta = Page(metaPg);
        if (!meta || meta[PAGE_TYPE] != P_BTREEMETA) return Fail(err, "bad meta page");
        std::set<uint32_t> seen;
        return Walk(U32(meta + META_ROOT), 0, seen, out, err);
    }
    bool HasSubdbs() const { return U32(P0() + META_FLAGS) & BTM_SUBDB; }

private:
    const unsigned char* P0() const { return reinterpret_cast<const unsigned char*>(f.data()); }
    const unsigned char* Page(uint32_t pg) const {
        if (pg >= npages) return nullptr;
        return P0() + (size_t)pg * pagesize;
    }
    static bool Fail(std::string& err, const char* what) {
        err = what;
        return false;
    }
    // item i of a page: its offset, checked to leave `need` bytes inside the page
    const unsigned char* Item(const unsigned char* page, unsigned i, size_t need) const {
        const unsigned n = U16(page + PAGE_ENTRIES);
        if (i >= n || PAGE_HDR + 2 * (size_t)(i + 1) > pagesize) return nullptr;
        const unsigned off = U16(page + PAGE_HDR + 2 * i);
        if (off < PAGE_HDR || off + need > pagesize) return nullptr;
        return page + off;
    }
    // a leaf item's bytes (inline or an overflow chain); false on a malformed item
    bool ItemBytes(const unsigned char* page, unsigned i, std::string& v, bool& deleted, std::string& err) const {
        const unsigned char* it = Item(page, i, 3);
        if (!it) return Fail(err, "bad leaf item offset");
        deleted = (it[2] & B_DELETE) != 0;
        const uint8_t type = it[2] & 0x7f;
        if (type == B_KEYDATA) {
            const uint16_t len = U16(it);
            if (!Item(page, i, 3 + (size_t)len)) return Fail(err, "leaf item past the page end");
            v.assign(reinterpret_cast<const char*>(it + 3), len);
            return true;
        }
        if (type == B_OVERFLOW) {
            if (!Item(page, i, 12)) return Fail(err, "overflow item past the page end");
            uint32_t pg = U32(it + 4);
            const uint32_t tlen = U32(it + 8);
            v.clear();
            std::set<uint32_t> chain;
            while (v.size() < tlen) {
                const unsigned char* op = Page(pg);
                if (!op || op[PAGE_TYPE] != P_OVERFLOW || !chain.insert(pg).second)
                    return Fail(err, "broken overflow chain");
                const uint16_t len = U16(op + PAGE_HFOFF);
                if (PAGE_HDR + (size_t)len > pagesize) return Fail(err, "overflow page length");
                v.append(reinterpret_cast<const char*>(op + PAGE_HDR), len);
                pg = U32(op + PAGE_NEXT);
            }
            if (v.size() != tlen) return Fail(err, "overflow chain length mismatch");
            return true;
        }
        return Fail(err, "unsupported leaf item type (duplicates)");
    }
    bool Walk(uint32_t pg, int depth, std::set<uint32_t>& seen, BdbRecords& out, std::string& err) {
        if (depth > 32 || !seen.insert(pg).second) return Fail(err, "btree cycle or depth");
        const unsigned char* page = Page(pg);
        if (!page) return Fail(err, "btree page beyond the end");
        const unsigned n = U16(page + PAGE_ENTRIES);
        if (page[PAGE_TYPE] == P_IBTREE) {
            for (unsigned i = 0; i < n; i++) {
                const unsigned char* it = Item(page, i, 12);
                if (!it) return Fail(err, "bad internal item");
                if (!Walk(U32(it + 4), depth + 1, seen, out, err)) return false;
            }
            return true;
        }
        if (page[PAGE_TYPE] != P_LBTREE) return Fail(err, "unexpected btree page type");
        if (n % 2) return Fail(err, "odd item count on a leaf page");
        for (unsigned i = 0; i < n; i += 2) {
            std::string k, v;
            bool dk = false, dv = false;
            if (!ItemBytes(page, i, k, dk, err) || !ItemBytes(page, i + 1, v, dv, err)) return false;
            if (!dk && !dv) out.emplace_back(std::move(k), std::move(v));
        }
        return true;
    }

    std::string f;
    size_t pagesize = 0, npages = 0;
};

bool ReadFile(const std::string& path, std::string& out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    out.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    return true;
}

bool FromHex(const std::string& s, std::string& out) {
    auto nib = [](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    };
    if (s.size() % 2) return false;
    out.resize(s.size() / 2);
    for (size_t i = 0; i < out.size(); i++) {
        const int hi = nib(s[2 * i]), lo = nib(s[2 * i + 1]);
        if (hi < 0 || lo < 0) return false;
        out[i] = (char)(hi * 16 + lo);
    }
    return true;
}

} // namespace

std::string BdbFileKind(const std::string& path) {
    struct stat st;
    if (stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return "";
    std::ifstream in(path, std::ios::binary);
    char head[16] = {};
    in.read(head, sizeof(head));
    if (in.gcount() >= 16 && U32(reinterpret_cast<const unsigned char*>(head) + META_MAGIC) == BTREE_MAGIC) return "btree";
    if (in.gcount() >= 8 && std::string(head, 8) == "VERSION=") return "dump";
    return "";
}

bool ReadBdbBtree(const std::string& path, BdbRecords& out, std::string& err) {
    std::string bytes;
    if (!ReadFile(path, bytes)) {
        err = "cannot read " + path;
        return false;
    }
    BtreeFile bf(std::move(bytes));
    if (!bf.Open(err)) return false;
    BdbRecords master;
    if (!bf.Records(0, master, err)) return false;
    if (!bf.HasSubdbs()) {
        out = std::move(master);
        return true;
    }
    // the master database maps sub-database names to their meta pages
    for (const auto& kv : master) {
        if (kv.first != "main") continue;
        if (kv.second.size() != 4) {
            err = "bad sub-database entry";
            return false;
        }
        return bf.Records(U32(reinterpret_cast<const unsigned char*>(kv.second.data())), out, err);
    }
    err = "no \"main\" sub-database";
    return false;
}

bool ReadBdbDump(std::istream& in, BdbRecords& out, std::string& err) {
    std::string line;
    bool header = true;
    std::string key;
    bool haveKey = false;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (header) {
            if (line == "HEADER=END") header = false;
            continue;
        }
        if (line == "DATA=END") {
            if (haveKey) {
                err = "dump: a key without a value";
                return false;
            }
            return true;
        }
        // data lines start with one space (db_dump -p would print text; only bytevalue is read)
        const size_t b = line.find_first_not_of(' ');
        std::string bytes;
        if (!FromHex(b == std::string::npos ? std::string() : line.substr(b), bytes)) {
            err = "dump: line is not hexadecimal (only the bytevalue format is read)";
            return false;
        }
        if (!haveKey) {
            key = std::move(bytes);
            haveKey = true;
        } else {
            out.emplace_back(std::move(key), std::move(bytes));
            haveKey = false;
        }
    }
    err = header ? "dump: no HEADER=END" : "dump: no DATA=END";
    return false;
}

} // namespace bcp

#include "node/kvstore.h"
#include "crypto/common.h"
#include "primitives/serialize.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <cstdio>
#include <filesystem>

namespace bcp {

namespace {
// The reference stores an unencrypted wallet key ("key" record) as the DER SEC1 ECPrivateKey
// its CKey::GetPrivKey exports (src/key.cpp ec_privkey_export_der: SEQUENCE { INTEGER 1,
// OCTET STRING secret, [0] curve parameters, [1] public key }), optionally followed by a hash;
// this wallet stores the 32-byte secret. The secret is the OCTET STRING after the version.
bool Sec1Secret(const std::vector<unsigned char>& der, std::vector<unsigned char>& secret) {
    size_t p = 0;
    const size_t n = der.size();
    auto len = [&](size_t& out) -> bool {
        if (p >= n) return false;
        const unsigned b = der[p++];
        if (b < 0x80) {
            out = b;
            return true;
        }
        const unsigned k = b & 0x7f;
        if (k == 0 || k > 2 || p + k > n) return false;
        out = 0;
        for (unsigned i = 0; i < k; i++) out = (out << 8) | der[p++];
        return true;
    };
    size_t l = 0;
    if (p >= n || der[p++] != 0x30 || !len(l) || p + l > n) return false;
    if (p + 3 > n || der[p] != 0x02 || der[p + 1] != 0x01 || der[p + 2] != 0x01) return false;
    p += 3;
    if (p >= n || der[p++] != 0x04 || !len(l) || l == 0 || l > 32 || p + l > n) return false;
    secret.assign(32 - l, 0);
    secret.insert(secret.end(), der.begin() + p, der.begin() + p + l);
    return true;
}

// A "key" record's value in this wallet's form (the 32-byte secret); other records unchanged.
void ConvertRecord(const std::string& key, std::string& value) {
    std::string type;
    try {
        SpanReader r((const unsigned char*)key.data(), key.size(), SER_DISK, PROTOCOL_VERSION);
        r >> type;
        if (type != "key") return;
        SpanReader v((const unsigned char*)value.data(), value.size(), SER_DISK, PROTOCOL_VERSION);
        std::vector<unsigned char> der, secret;
        v >> der;
        if (der.size() == 32 || !Sec1Secret(der, secret)) return; // already a bare secret, or unknown
        std::vector<unsigned char> out;
        VectorWriter w(out, SER_DISK, PROTOCOL_VERSION);
        w << secret;
        value.assign(out.begin(), out.end());
        memory_cleanse(secret.data(), secret.size());
        memory_cleanse(der.data(), der.size());
    } catch (const std::exception&) {
    }
}
} // namespace

bool ImportBdbWalletFile(const std::string& path, size_t& imported, std::string& err) {
    const std::string kind = BdbFileKind(path);
    BdbRecords recs;
    if (kind == "btree") {
        if (!ReadBdbBtree(path, recs, err)) return false;
    } else if (kind == "dump") {
        std::ifstream in(path);
        if (!ReadBdbDump(in, recs, err)) return false;
    } else {
        err = path + " is not a Berkeley DB wallet";
        return false;
    }
    // Build the converted store beside the original and only then swap: a failed write, or a
    // process that dies before the renames, leaves wallet.dat untouched (and the next start
    // imports it again) instead of an empty native store at the wallet path.
    const std::string tmp = path + ".import.tmp";
    std::error_code ec;
    std::filesystem::remove_all(tmp, ec);
    bool written = false;
    {
        KVStore fresh(tmp, false, true);
        KVBatch b;
        for (auto& kv : recs) {
            ConvertRecord(kv.first, kv.second);
            b.WriteRaw(kv.first, kv.second);
        }
        written = fresh.WriteBatch(b, true);
    }
    // the records (plaintext key material among them) are not needed past the batch
    for (auto& kv : recs) {
        memory_cleanse(&kv.second[0], kv.second.size());
        memory_cleanse(&kv.first[0], kv.first.size());
    }
    if (!written) {
        std::filesystem::remove_all(tmp, ec);
        err = "writing the imported wallet failed";
        return false;
    }
    const std::string bak = strprintf("%s.bdb.%lld", path.c_str(), (long long)GetTime());
    if (rename(path.c_str(), bak.c_str()) != 0) {
        std::filesystem::remove_all(tmp, ec);
        err = "cannot move " + path + " aside to " + bak;
        return false;
    }
    if (rename(tmp.c_str(), path.c_str()) != 0) {
        rename(bak.c_str(), path.c_str()); // put the original back
        std::filesystem::remove_all(tmp, ec);
        err = "cannot move the imported wallet into place at " + path;
        return false;
    }
    imported = recs.size();
    LogPrintf("Imported %u records from the Berkeley DB wallet %s (original kept as %s)\n", (unsigned)recs.size(),
              path.c_str(), bak.c_str());
    return true;
}

} // namespace bcp
