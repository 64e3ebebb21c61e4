// Binary serialisation: little-endian integers, CompactSize, VarInt, containers,
// plus in-memory streams and a SHA-256d hashing stream.
// Wire-format parity: reference src/serialize.h:370-894 (CompactSize, VarInt,
// vector/string/pair) and src/streams.h (CDataStream), src/hash.h:136 (CHashWriter).
// Design: a small set of free functions dispatching to member Serialize/Unserialize;
// no READWRITE macro machinery.
#pragma once
#include "util/prevector.h"
#include "crypto/hashes.h"
#include "primitives/uint256.h"

#include <cstdint>
#include <cstring>
#include <ios>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace bcp {

static const unsigned int MAX_SIZE = 0x02000000; // 32 MiB, reference src/serialize.h:25

enum SerType { SER_NETWORK = (1 << 0), SER_DISK = (1 << 1), SER_GETHASH = (1 << 2) };

// Peer/stream protocol versions (reference src/version.h:11-50).
static const int PROTOCOL_VERSION = 70016;
static const int BCP_HARD_FORK_VERSION = 70016;
static const int INIT_PROTO_VERSION = 209;
static const int MIN_PEER_PROTO_VERSION = 31800;
static const int SENDHEADERS_VERSION = 70012;
static const int FEEFILTER_VERSION = 70013;
static const int SHORT_IDS_BLOCKS_VERSION = 70014;
static const int NO_BLOOM_VERSION = 70011;
static const int BIP0031_VERSION = 60000;
static const int CADDR_TIME_VERSION = 31402;
// Stream-version flag selecting the 80-byte legacy block header (reference src/primitives/block.h:20).
static const int SERIALIZE_BLOCK_LEGACY = 0x04000000;
static const int SERIALIZE_TRANSACTION_NO_WITNESS = 0x40000000;

class ser_error : public std::ios_base::failure {
public:
    explicit ser_error(const std::string& m) : std::ios_base::failure(m) {}
};

// ---------------------------------------------------------------- primitives
// Tag selecting stream-deserialising constructors, e.g. CTransaction(deserialize, stream).
struct deserialize_type {};
constexpr deserialize_type deserialize{};

template <typename S> inline void ser_u8(S& s, uint8_t v) { s.write((const char*)&v, 1); }
template <typename S> inline void ser_u16(S& s, uint16_t v) { s.write((const char*)&v, 2); }
template <typename S> inline void ser_u32(S& s, uint32_t v) { s.write((const char*)&v, 4); }
template <typename S> inline void ser_u64(S& s, uint64_t v) { s.write((const char*)&v, 8); }
template <typename S> inline uint8_t unser_u8(S& s) { uint8_t v; s.read((char*)&v, 1); return v; }
template <typename S> inline uint16_t unser_u16(S& s) { uint16_t v; s.read((char*)&v, 2); return v; }
template <typename S> inline uint32_t unser_u32(S& s) { uint32_t v; s.read((char*)&v, 4); return v; }
template <typename S> inline uint64_t unser_u64(S& s) { uint64_t v; s.read((char*)&v, 8); return v; }

inline unsigned int GetSizeOfCompactSize(uint64_t n) {
    if (n < 253) return 1;
    if (n <= 0xFFFF) return 3;
    if (n <= 0xFFFFFFFFu) return 5;
    return 9;
}

template <typename S> void WriteCompactSize(S& s, uint64_t n) {
    if (n < 253) {
        ser_u8(s, (uint8_t)n);
    } else if (n <= 0xFFFF) {
        ser_u8(s, 253);
        ser_u16(s, (uint16_t)n);
    } else if (n <= 0xFFFFFFFFu) {
        ser_u8(s, 254);
        ser_u32(s, (uint32_t)n);
    } else {
        ser_u8(s, 255);
        ser_u64(s, n);
    }
}

template <typename S> uint64_t ReadCompactSize(S& s, bool range_check = true) {
    uint8_t chSize = unser_u8(s);
    uint64_t n;
    if (chSize < 253) {
        n = chSize;
    } else if (chSize == 253) {
        n = unser_u16(s);
        if (n < 253) throw ser_error("non-canonical ReadCompactSize()");
    } else if (chSize == 254) {
        n = unser_u32(s);
        if (n < 0x10000u) throw ser_error("non-canonical ReadCompactSize()");
    } else {
        n = unser_u64(s);
        if (n < 0x100000000ULL) throw ser_error("non-canonical ReadCompactSize()");
    }
    if (range_check && n > (uint64_t)MAX_SIZE) throw ser_error("ReadCompactSize(): size too large");
    return n;
}

// Bitcoin "VarInt": MSB base-128 with an offset of one per continuation byte
// (reference src/serialize.h WriteVarInt/ReadVarInt). Used by the UTXO/undo formats.
template <typename S> void WriteVarInt(S& s, uint64_t n) {
    unsigned char tmp[(sizeof(n) * 8 + 6) / 7];
    int len = 0;
    while (true) {
        tmp[len] = (n & 0x7F) | (len ? 0x80 : 0x00);
        if (n <= 0x7F) break;
        n = (n >> 7) - 1;
        len++;
    }
    do { ser_u8(s, tmp[len]); } while (len--);
}

template <typename S> uint64_t ReadVarInt(S& s) {
    uint64_t n = 0;
    while (true) {
        unsigned char chData = unser_u8(s);
        if (n > (std::numeric_limits<uint64_t>::max() >> 7)) throw ser_error("ReadVarInt(): size too large");
        n = (n << 7) | (chData & 0x7F);
        if (chData & 0x80) {
            if (n == std::numeric_limits<uint64_t>::max()) throw ser_error("ReadVarInt(): size too large");
            n++;
        } else {
            return n;
        }
    }
}

// ---------------------------------------------------------------- dispatch
template <typename S> inline void Serialize(S& s, bool v) { ser_u8(s, v ? 1 : 0); }
template <typename S> inline void Serialize(S& s, char v) { ser_u8(s, (uint8_t)v); }
template <typename S> inline void Serialize(S& s, int8_t v) { ser_u8(s, (uint8_t)v); }
template <typename S> inline void Serialize(S& s, uint8_t v) { ser_u8(s, v); }
template <typename S> inline void Serialize(S& s, int16_t v) { ser_u16(s, (uint16_t)v); }
template <typename S> inline void Serialize(S& s, uint16_t v) { ser_u16(s, v); }
template <typename S> inline void Serialize(S& s, int32_t v) { ser_u32(s, (uint32_t)v); }
template <typename S> inline void Serialize(S& s, uint32_t v) { ser_u32(s, v); }
template <typename S> inline void Serialize(S& s, int64_t v) { ser_u64(s, (uint64_t)v); }
template <typename S> inline void Serialize(S& s, uint64_t v) { ser_u64(s, v); }

template <typename S> inline void Unserialize(S& s, bool& v) { v = unser_u8(s) != 0; }
template <typename S> inline void Unserialize(S& s, char& v) { v = (char)unser_u8(s); }
template <typename S> inline void Unserialize(S& s, int8_t& v) { v = (int8_t)unser_u8(s); }
template <typename S> inline void Unserialize(S& s, uint8_t& v) { v = unser_u8(s); }
template <typename S> inline void Unserialize(S& s, int16_t& v) { v = (int16_t)unser_u16(s); }
template <typename S> inline void Unserialize(S& s, uint16_t& v) { v = unser_u16(s); }
template <typename S> inline void Unserialize(S& s, int32_t& v) { v = (int32_t)unser_u32(s); }
template <typename S> inline void Unserialize(S& s, uint32_t& v) { v = unser_u32(s); }
template <typename S> inline void Unserialize(S& s, int64_t& v) { v = (int64_t)unser_u64(s); }
template <typename S> inline void Unserialize(S& s, uint64_t& v) { v = unser_u64(s); }

// class types with member functions
template <typename S, typename T>
inline auto Serialize(S& s, const T& obj) -> decltype(obj.Serialize(s), void()) { obj.Serialize(s); }
template <typename S, typename T>
inline auto Unserialize(S& s, T& obj) -> decltype(obj.Unserialize(s), void()) { obj.Unserialize(s); }

// strings
template <typename S> void Serialize(S& s, const std::string& str) {
    WriteCompactSize(s, str.size());
    if (!str.empty()) s.write(str.data(), str.size());
}
template <typename S> void Unserialize(S& s, std::string& str) {
    uint64_t n = ReadCompactSize(s);
    str.resize(n);
    if (n) s.read(&str[0], n);
}

// prevector (script bytes): like a byte vector
template <typename S, unsigned N, typename T> void Serialize(S& s, const prevector<N, T>& v) {
    static_assert(sizeof(T) == 1, "byte prevectors only");
    WriteCompactSize(s, v.size());
    if (!v.empty()) s.write((const char*)v.data(), v.size());
}
template <typename S, unsigned N, typename T> void Unserialize(S& s, prevector<N, T>& v) {
    static_assert(sizeof(T) == 1, "byte prevectors only");
    v.clear();
    const uint64_t n = ReadCompactSize(s);
    // in chunks, so a lying length prefix cannot force a huge allocation
    uint64_t i = 0;
    while (i < n) {
        const uint64_t blk = std::min<uint64_t>(n - i, 5000000);
        v.resize((uint32_t)(i + blk));
        s.read((char*)v.data() + i, blk);
        i += blk;
    }
}

// vectors: byte vectors are raw, others element-wise
template <typename S, typename T, typename A> void Serialize(S& s, const std::vector<T, A>& v);
template <typename S, typename T, typename A> void Unserialize(S& s, std::vector<T, A>& v);
template <typename S, typename K, typename V> void Serialize(S& s, const std::pair<K, V>& p);
template <typename S, typename K, typename V> void Unserialize(S& s, std::pair<K, V>& p);
template <typename S, typename T> void Serialize(S& s, const std::shared_ptr<const T>& p);
template <typename S, typename T> void Unserialize(S& s, std::shared_ptr<const T>& p);

template <typename S, typename T, typename A> void Serialize(S& s, const std::vector<T, A>& v) {
    WriteCompactSize(s, v.size());
    if constexpr (std::is_same<T, unsigned char>::value || std::is_same<T, char>::value) {
        if (!v.empty()) s.write((const char*)v.data(), v.size());
    } else {
        for (const auto& e : v) Serialize(s, e);
    }
}
template <typename S, typename T, typename A> void Unserialize(S& s, std::vector<T, A>& v) {
    v.clear();
    uint64_t n = ReadCompactSize(s);
    if constexpr (std::is_same<T, unsigned char>::value || std::is_same<T, char>::value) {
        // Read in chunks so a lying length prefix cannot force a huge allocation.
        uint64_t i = 0;
        while (i < n) {
            uint64_t blk = std::min<uint64_t>(n - i, 1 + 4999999 / sizeof(T));
            v.resize(i + blk);
            s.read((char*)&v[i], blk);
            i += blk;
        }
    } else {
        uint64_t i = 0, nMid = 0;
        while (nMid < n) {
            nMid += 5000000 / sizeof(T);
            if (nMid > n) nMid = n;
            v.resize(nMid);
            for (; i < nMid; i++) Unserialize(s, v[i]);
        }
    }
}
template <typename S, typename K, typename V> void Serialize(S& s, const std::pair<K, V>& p) {
    Serialize(s, p.first);
    Serialize(s, p.second);
}
template <typename S, typename K, typename V> void Unserialize(S& s, std::pair<K, V>& p) {
    Unserialize(s, p.first);
    Unserialize(s, p.second);
}
template <typename S, typename K, typename V, typename C> void Serialize(S& s, const std::map<K, V, C>& m) {
    WriteCompactSize(s, m.size());
    for (const auto& kv : m) { Serialize(s, kv.first); Serialize(s, kv.second); }
}
template <typename S, typename K, typename V, typename C> void Unserialize(S& s, std::map<K, V, C>& m) {
    m.clear();
    uint64_t n = ReadCompactSize(s);
    for (uint64_t i = 0; i < n; i++) {
        K k; V v;
        Unserialize(s, k);
        Unserialize(s, v);
        m.emplace(std::move(k), std::move(v));
    }
}
template <typename S, typename K, typename C> void Serialize(S& s, const std::set<K, C>& m) {
    WriteCompactSize(s, m.size());
    for (const auto& k : m) Serialize(s, k);
}
template <typename S, typename K, typename C> void Unserialize(S& s, std::set<K, C>& m) {
    m.clear();
    uint64_t n = ReadCompactSize(s);
    for (uint64_t i = 0; i < n; i++) { K k; Unserialize(s, k); m.insert(std::move(k)); }
}
template <typename S, typename T> void Serialize(S& s, const std::shared_ptr<const T>& p) { Serialize(s, *p); }
template <typename S, typename T> void Unserialize(S& s, std::shared_ptr<const T>& p) {
    p = std::make_shared<const T>(deserialize, s);  // T(deserialize_type, S&) constructor
}

// Fixed-size array of POD bytes
template <typename S, size_t N> void Serialize(S& s, const unsigned char (&a)[N]) { s.write((const char*)a, N); }
template <typename S, size_t N> void Unserialize(S& s, unsigned char (&a)[N]) { s.read((char*)a, N); }

// Wrapper for VarInt-encoded fields and compact-size fields.
template <typename I> struct VarIntRef {
    I& n;
    template <typename S> void Serialize(S& s) const { WriteVarInt(s, (uint64_t)n); }
    template <typename S> void Unserialize(S& s) { n = (I)ReadVarInt(s); }
};
template <typename I> VarIntRef<I> VARINT(I& n) { return VarIntRef<I>{n}; }
template <typename I> VarIntRef<I> VARINT(const I& n) { return VarIntRef<I>{const_cast<I&>(n)}; }

// ---------------------------------------------------------------- streams
class SizeComputer {
    size_t nSize = 0;
    int nVersion;
public:
    explicit SizeComputer(int v) : nVersion(v) {}
    void write(const char*, size_t n) { nSize += n; }
    void read(char*, size_t) { throw ser_error("SizeComputer read"); }
    size_t size() const { return nSize; }
    int GetVersion() const { return nVersion; }
    int GetType() const { return 0; }
    void seek(size_t n) { nSize += n; }
};

template <typename T> size_t GetSerializeSize(const T& t, int nVersion = PROTOCOL_VERSION) {
    SizeComputer sc(nVersion);
    Serialize(sc, t);
    return sc.size();
}

// Growable byte buffer with a read cursor (CDataStream equivalent).
class DataStream {
    std::vector<char> vch;
    size_t nReadPos = 0;
    int nType, nVersion;
public:
    DataStream(int type = SER_NETWORK, int version = PROTOCOL_VERSION) : nType(type), nVersion(version) {}
    DataStream(const std::vector<unsigned char>& v, int type = SER_NETWORK, int version = PROTOCOL_VERSION)
        : vch(v.begin(), v.end()), nType(type), nVersion(version) {}
    DataStream(const char* b, const char* e, int type = SER_NETWORK, int version = PROTOCOL_VERSION)
        : vch(b, e), nType(type), nVersion(version) {}
    int GetType() const { return nType; }
    int GetVersion() const { return nVersion; }
    void SetVersion(int v) { nVersion = v; }
    void SetType(int t) { nType = t; }
    size_t size() const { return vch.size() - nReadPos; }
    bool empty() const { return size() == 0; }
    bool eof() const { return size() == 0; }
    const char* data() const { return vch.data() + nReadPos; }
    char* data() { return vch.data() + nReadPos; }
    void clear() { vch.clear(); nReadPos = 0; }
    void reserve(size_t n) { vch.reserve(n); }
    void write(const char* p, size_t n) { vch.insert(vch.end(), p, p + n); }
    void read(char* p, size_t n) {
        if (n == 0) return;
        if (nReadPos + n > vch.size()) throw ser_error("DataStream::read(): end of data");
        if (n) memcpy(p, vch.data() + nReadPos, n);
        nReadPos += n;
        if (nReadPos == vch.size()) { nReadPos = 0; vch.clear(); }
    }
    void ignore(size_t n) {
        if (nReadPos + n > vch.size()) throw ser_error("DataStream::ignore(): end of data");
        nReadPos += n;
        if (nReadPos == vch.size()) { nReadPos = 0; vch.clear(); }
    }
    void Rewind(size_t n) {
        if (n > nReadPos) throw ser_error("DataStream::Rewind out of range");
        nReadPos -= n;
    }
    std::vector<unsigned char> Bytes() const { return std::vector<unsigned char>(vch.begin() + nReadPos, vch.end()); }
    std::string str() const { return std::string(vch.begin() + nReadPos, vch.end()); }
    template <typename T> DataStream& operator<<(const T& obj) { ::bcp::Serialize(*this, obj); return *this; }
    template <typename T> DataStream& operator>>(T& obj) { ::bcp::Unserialize(*this, obj); return *this; }
    DataStream& operator<<(const VarIntRef<uint64_t>& v) { v.Serialize(*this); return *this; }
};

// Reader over a caller-owned span; never copies.
class SpanReader {
    const unsigned char* p;
    size_t n, pos = 0;
    int nType, nVersion;
public:
    SpanReader(const unsigned char* data, size_t len, int type = SER_NETWORK, int version = PROTOCOL_VERSION)
        : p(data), n(len), nType(type), nVersion(version) {}
    int GetType() const { return nType; }
    int GetVersion() const { return nVersion; }
    void read(char* dst, size_t k) {
        if (pos + k > n) throw ser_error("SpanReader::read(): end of data");
        if (k == 0) return; // an empty vector's data() may be null: memcpy(null, ..., 0) is UB
        memcpy(dst, p + pos, k);
        pos += k;
    }
    void ignore(size_t k) {
        if (k > n - pos) throw ser_error("SpanReader::ignore(): end of data");
        pos += k;
    }
    size_t size() const { return n - pos; }
    bool empty() const { return pos == n; }
    size_t tell() const { return pos; }
    template <typename T> SpanReader& operator>>(T& obj) { ::bcp::Unserialize(*this, obj); return *this; }
};

// Appends into a caller vector (CVectorWriter equivalent).
class VectorWriter {
    std::vector<unsigned char>& v;
    int nType, nVersion;
public:
    VectorWriter(std::vector<unsigned char>& out, int type = SER_NETWORK, int version = PROTOCOL_VERSION)
        : v(out), nType(type), nVersion(version) {}
    int GetType() const { return nType; }
    int GetVersion() const { return nVersion; }
    void write(const char* p, size_t k) { v.insert(v.end(), (const unsigned char*)p, (const unsigned char*)p + k); }
    template <typename T> VectorWriter& operator<<(const T& obj) { ::bcp::Serialize(*this, obj); return *this; }
};

// SHA-256d over everything written (CHashWriter).
class HashWriter {
    CSHA256 ctx;
    int nType, nVersion;
    size_t nBytes = 0;
public:
    HashWriter(int type = SER_GETHASH, int version = PROTOCOL_VERSION) : nType(type), nVersion(version) {}
    int GetType() const { return nType; }
    int GetVersion() const { return nVersion; }
    void write(const char* p, size_t n) {
        ctx.Write((const unsigned char*)p, n);
        nBytes += n;
    }
    size_t BytesWritten() const { return nBytes; }
    uint256 GetHash() {
        uint256 r;
        ctx.Finalize(r.begin());
        CSHA256().Write(r.begin(), 32).Finalize(r.begin());
        return r;
    }
    uint256 GetSHA256() { uint256 r; ctx.Finalize(r.begin()); return r; }
    template <typename T> HashWriter& operator<<(const T& obj) { ::bcp::Serialize(*this, obj); return *this; }
};

template <typename T> uint256 SerializeHash(const T& obj, int type = SER_GETHASH, int version = PROTOCOL_VERSION) {
    HashWriter hw(type, version);
    hw << obj;
    return hw.GetHash();
}

template <typename T> std::vector<unsigned char> SerializeToBytes(const T& obj, int type = SER_NETWORK,
                                                                  int version = PROTOCOL_VERSION) {
    std::vector<unsigned char> out;
    VectorWriter w(out, type, version);
    w << obj;
    return out;
}

inline uint256 Hash256(const unsigned char* p, size_t n) { uint256 r; Sha256d(p, n, r.begin()); return r; }
inline uint256 Hash256(const std::vector<unsigned char>& v) { return Hash256(v.data(), v.size()); }
inline uint256 Hash256Concat(const uint256& a, const uint256& b) {
    unsigned char buf[64];
    memcpy(buf, a.begin(), 32);
    memcpy(buf + 32, b.begin(), 32);
    return Hash256(buf, 64);
}
inline uint160 Hash160(const std::vector<unsigned char>& v) {
    uint160 r;
    ::bcp::Hash160(v.data(), v.size(), r.begin());
    return r;
}
template <unsigned N> inline uint160 Hash160(const prevector<N, unsigned char>& v) {
    uint160 r;
    ::bcp::Hash160(v.data(), v.size(), r.begin());
    return r;
}

} // namespace bcp
