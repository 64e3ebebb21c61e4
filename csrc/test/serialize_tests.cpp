// Wire/disk serialization primitives, streams and the UTXO compression formats.
// Parity: reference src/test/serialize_tests.cpp (sizes, varints, varints_bitpatterns,
// compactsize, noncanonical, class_methods), src/test/streams_tests.cpp (vector writer, empty
// vectors) and src/test/compress_tests.cpp (compress_amounts). Round trips are checked over
// generated value sweeps; byte patterns are the format's fixed encodings.
#include "node/coins.h"
#include "primitives/serialize.h"
#include "script/standard.h"
#include "test/unittest.h"
#include "util/strencodings.h"

#include <limits>
#include <map>

namespace bcp {
namespace {

template <typename T> std::string Ser(const T& v) {
    DataStream s;
    s << v;
    return HexStr(s.Bytes());
}
std::string VarIntHex(uint64_t n) {
    std::vector<unsigned char> out;
    VectorWriter w(out);
    WriteVarInt(w, n);
    return HexStr(out);
}

struct Record {
    int32_t a = 0;
    bool b = false;
    std::string c;
    std::vector<uint16_t> d;
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, a);
        ::bcp::Serialize(s, b);
        ::bcp::Serialize(s, c);
        ::bcp::Serialize(s, d);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, a);
        ::bcp::Unserialize(s, b);
        ::bcp::Unserialize(s, c);
        ::bcp::Unserialize(s, d);
    }
    bool operator==(const Record& o) const { return a == o.a && b == o.b && c == o.c && d == o.d; }
};

} // namespace

TEST_CASE(serialize_tests, sizes) {
    CHECK_EQ(GetSerializeSize(char(0)), (size_t)1);
    CHECK_EQ(GetSerializeSize(int8_t(0)), (size_t)1);
    CHECK_EQ(GetSerializeSize(uint16_t(0)), (size_t)2);
    CHECK_EQ(GetSerializeSize(int32_t(0)), (size_t)4);
    CHECK_EQ(GetSerializeSize(uint32_t(0)), (size_t)4);
    CHECK_EQ(GetSerializeSize(int64_t(0)), (size_t)8);
    CHECK_EQ(GetSerializeSize(uint64_t(0)), (size_t)8);
    CHECK_EQ(GetSerializeSize(true), (size_t)1);
    CHECK_EQ(GetSerializeSize(std::string(300, 'x')), (size_t)303); // 3-byte length prefix
    CHECK_EQ(GetSerializeSize(std::vector<uint32_t>(10)), (size_t)41);
    // integers are little-endian
    CHECK_EQ(Ser(uint32_t(0x01020304)), std::string("04030201"));
    CHECK_EQ(Ser(int16_t(-2)), std::string("feff"));
    CHECK_EQ(Ser(uint64_t(1) << 40), std::string("0000000000010000"));
}

TEST_CASE(serialize_tests, varints) {
    // round trip over values spread across every magnitude, sizes as the size computer says
    std::vector<unsigned char> buf;
    VectorWriter w(buf);
    std::vector<uint64_t> vals;
    for (int shift = 0; shift < 64; shift++)
        for (uint64_t d : {0ULL, 1ULL, 0x7FULL, 0x80ULL}) vals.push_back((1ULL << shift) + d - (shift ? 1 : 0));
    vals.push_back(std::numeric_limits<uint64_t>::max());
    size_t total = 0;
    for (uint64_t v : vals) {
        WriteVarInt(w, v);
        SizeComputer sc(PROTOCOL_VERSION);
        WriteVarInt(sc, v);
        total += sc.size();
    }
    CHECK_EQ(buf.size(), total);
    SpanReader r(buf.data(), buf.size());
    for (uint64_t v : vals) CHECK_EQ(ReadVarInt(r), v);
    CHECK(r.empty());
    // the format's fixed encodings (base 128, MSB first, one subtracted per continuation)
    CHECK_EQ(VarIntHex(0), std::string("00"));
    CHECK_EQ(VarIntHex(0x7f), std::string("7f"));
    CHECK_EQ(VarIntHex(0x80), std::string("8000"));
    CHECK_EQ(VarIntHex(0x1234), std::string("a334"));
    CHECK_EQ(VarIntHex(0xffff), std::string("82fe7f"));
    CHECK_EQ(VarIntHex(0xffffffffULL), std::string("8efefefe7f"));
    CHECK_EQ(VarIntHex(std::numeric_limits<uint64_t>::max()), std::string("80fefefefefefefefe7f"));
    // an encoding that overflows 64 bits is refused
    std::vector<unsigned char> big = ParseHex("80fefefefefefefefefe7f");
    SpanReader rb(big.data(), big.size());
    CHECK_THROWS(ReadVarInt(rb));
}

TEST_CASE(serialize_tests, compactsize) {
    // every boundary of the 1/3/5/9-byte forms round-trips with the predicted size
    std::vector<uint64_t> vals{0, 1, 252, 253, 254, 0xFFFF, 0x10000, 0xFFFFFFFFULL, 0x100000000ULL};
    for (uint64_t v : vals) {
        std::vector<unsigned char> b;
        VectorWriter w(b);
        WriteCompactSize(w, v);
        CHECK_EQ(b.size(), (size_t)GetSizeOfCompactSize(v));
        SpanReader r(b.data(), b.size());
        CHECK_EQ(ReadCompactSize(r, false), v);
    }
    // sizes above MAX_SIZE are refused unless range checking is off
    std::vector<unsigned char> b;
    VectorWriter w(b);
    WriteCompactSize(w, (uint64_t)MAX_SIZE + 1);
    SpanReader r1(b.data(), b.size());
    CHECK_THROWS(ReadCompactSize(r1));
    // non-canonical forms (a longer encoding than needed) are refused
    const std::pair<const char*, bool> cases[] = {
        {"fdfc00", false},             // 252 in 3 bytes
        {"fdfd00", true},              // 253: the smallest 3-byte value
        {"feffff0000", false},         // 0xffff in 5 bytes
        {"fe00000100", true},          // 0x10000
        {"ffffffffff00000000", false}, // 0xffffffff in 9 bytes
        {"ff0000000001000000", true},  // 2^32
    };
    for (const auto& c : cases) {
        std::vector<unsigned char> v = ParseHex(c.first);
        SpanReader r(v.data(), v.size());
        if (c.second) {
            bool ok = true;
            try {
                ReadCompactSize(r, false);
            } catch (const std::exception&) {
                ok = false;
            }
            CHECK(ok);
        } else {
            CHECK_THROWS(ReadCompactSize(r, false));
        }
    }
}

TEST_CASE(serialize_tests, containers_and_classes) {
    Record a;
    a.a = -5;
    a.b = true;
    a.c = "serialize me";
    a.d = {1, 2, 65535};
    DataStream s;
    s << a;
    CHECK_EQ(s.size(), (size_t)(4 + 1 + 1 + 12 + 1 + 6));
    Record b;
    s >> b;
    CHECK(a == b);
    CHECK(s.empty());
    // reading past the end throws
    DataStream t;
    t << uint16_t(7);
    uint32_t x;
    CHECK_THROWS(t >> x);
    // maps, pairs, nested vectors
    std::map<std::string, std::vector<int64_t>> m{{"a", {1, -1}}, {"bb", {}}, {"c", {1LL << 62}}};
    DataStream u;
    u << m;
    std::map<std::string, std::vector<int64_t>> m2;
    u >> m2;
    CHECK(m == m2);
    // an empty vector serializes to its zero length alone, and reads back empty
    DataStream e;
    e << std::vector<unsigned char>();
    CHECK_EQ(HexStr(e.Bytes()), std::string("00"));
    std::vector<unsigned char> ev{9};
    e >> ev;
    CHECK(ev.empty());
}

TEST_CASE(streams_tests, vector_writer) {
    // appends after whatever the vector already holds
    std::vector<unsigned char> v{0xaa, 0xbb};
    VectorWriter w(v);
    w << uint8_t(1) << uint16_t(0x0302);
    CHECK_EQ(HexStr(v), std::string("aabb010203"));
    // the span reader never reads beyond its span and reports what is left
    SpanReader r(v.data() + 2, 3);
    uint8_t one;
    r >> one;
    CHECK_EQ((int)one, 1);
    CHECK_EQ(r.size(), (size_t)2);
    uint32_t too_big;
    CHECK_THROWS(r >> too_big);
    // rewinding a data stream re-reads the same bytes
    DataStream s;
    s << uint32_t(0xdeadbeef) << uint32_t(1);
    uint32_t x, y;
    s >> x;
    s.Rewind(4);
    s >> y;
    CHECK_EQ(x, y);
}

TEST_CASE(compress_tests, amounts) {
    // the amounts that matter compress to tiny numbers
    CHECK_EQ(CompressAmount(0), (uint64_t)0);
    CHECK_EQ(CompressAmount(1), (uint64_t)1);
    CHECK_EQ(CompressAmount(1000000), (uint64_t)7);         // 0.01 BCP
    CHECK_EQ(CompressAmount(100000000), (uint64_t)9);       // 1 BCP
    CHECK_EQ(CompressAmount(5000000000ULL), (uint64_t)50);  // 50 BCP
    CHECK_EQ(CompressAmount(2100000000000000ULL), (uint64_t)21000000);
    // round trips: every amount up to 200000 satoshi, and multiples at every power of ten
    for (uint64_t n = 0; n <= 200000; n++) CHECK_EQ(DecompressAmount(CompressAmount(n)), n);
    for (uint64_t p = 1; p <= 1000000000000000ULL; p *= 10)
        for (uint64_t k : {1ULL, 3ULL, 7ULL, 9ULL, 12ULL, 99ULL, 12345ULL})
            if (k * p <= 2100000000000000ULL) CHECK_EQ(DecompressAmount(CompressAmount(k * p)), k * p);
    // and the compressed space decodes uniquely
    for (uint64_t c = 0; c < 100000; c++) CHECK_EQ(CompressAmount(DecompressAmount(c)), c);
}

TEST_CASE(compress_tests, scripts) {
    // P2PKH, P2SH and pay-to-pubkey compress to their 21/33-byte special forms and back
    CKey key;
    key.MakeNewKey(true);
    const CPubKey pub = key.GetPubKey();
    CKey ukey;
    ukey.MakeNewKey(false);
    const CPubKey upub = ukey.GetPubKey();
    const CScript scripts[] = {
        GetScriptForDestination(pub.GetID()),
        GetScriptForDestination(CScriptID(GetScriptForDestination(pub.GetID()))),
        GetScriptForRawPubKey(pub),
        GetScriptForRawPubKey(upub),
    };
    const size_t sizes[] = {21, 21, 33, 33};
    for (int i = 0; i < 4; i++) {
        std::vector<unsigned char> c;
        CHECK(CompressScript(scripts[i], c));
        CHECK_EQ(c.size(), sizes[i]);
        DataStream s;
        SerializeCompressedScript(s, scripts[i]);
        CScript back;
        UnserializeCompressedScript(s, back);
        CHECK(back == scripts[i]);
    }
    // anything else is stored raw, behind its length + 6
    CScript other = CScript() << OP_RETURN << std::vector<unsigned char>(20, 7);
    std::vector<unsigned char> c;
    CHECK(!CompressScript(other, c));
    DataStream s;
    SerializeCompressedScript(s, other);
    CHECK_EQ(s.size(), other.size() + 1);
    CScript back;
    UnserializeCompressedScript(s, back);
    CHECK(back == other);
}

} // namespace bcp
