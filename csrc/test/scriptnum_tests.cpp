// scriptnum_tests: CScriptNum (csrc/script/script.h) against an independent reference number.
// Parity: reference src/test/scriptnum_tests.cpp (creation from int64 / from serialized
// bytes, +, -, unary -, the six comparisons, over a value x offset grid; serialized numbers
// longer than 4 bytes are refused). The reference compares against CScriptNum10 (the 0.10-era
// implementation); here the reference is a 128-bit integer with its own sign-magnitude
// little-endian codec and int32 saturation, written from the encoding rules, not from either
// implementation.
#include "test/unittest.h"

#include "script/script.h"

#include <cstdint>
#include <limits>
#include <vector>

using namespace bcp;

namespace {

// The reference model: exact value in __int128, minimal sign-magnitude little-endian bytes.
struct RefNum {
    __int128 v;
    explicit RefNum(__int128 x) : v(x) {}
    static RefNum FromBytes(const std::vector<unsigned char>& b, size_t maxSize = 4) {
        if (b.size() > maxSize) throw scriptnum_error("overflow");
        if (b.empty()) return RefNum(0);
        unsigned __int128 mag = 0;
        for (size_t i = 0; i < b.size(); i++) {
            unsigned char byte = b[i];
            if (i + 1 == b.size()) byte &= 0x7f; // the sign bit lives in the last byte
            mag |= (unsigned __int128)byte << (8 * i);
        }
        return RefNum((b.back() & 0x80) ? -(__int128)mag : (__int128)mag);
    }
    std::vector<unsigned char> Bytes() const {
        std::vector<unsigned char> out;
        if (v == 0) return out;
        const bool neg = v < 0;
        unsigned __int128 mag = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
        while (mag) {
            out.push_back((unsigned char)(mag & 0xff));
            mag >>= 8;
        }
        // the top bit of the last byte is the sign: add a byte when the magnitude uses it
        if (out.back() & 0x80) out.push_back(neg ? 0x80 : 0x00);
        else if (neg) out.back() |= 0x80;
        return out;
    }
    int Int() const {
        if (v > std::numeric_limits<int>::max()) return std::numeric_limits<int>::max();
        if (v < std::numeric_limits<int>::min()) return std::numeric_limits<int>::min();
        return (int)v;
    }
};

bool Same(const RefNum& r, const CScriptNum& s) { return r.Bytes() == s.getvch() && r.Int() == s.getint(); }

const int64_t VALUES[] = {0, 1, -2, 127, 128, -255, 256, (1LL << 15) - 1, -(1LL << 16), (1LL << 24) - 1, (1LL << 31),
                          1 - (1LL << 32), 1LL << 40};
const int64_t OFFSETS[] = {1, 0x79, 0x80, 0x81, 0xFF, 0x7FFF, 0x8000, 0xFFFF, 0x10000};
constexpr int64_t I64MAX = std::numeric_limits<int64_t>::max(), I64MIN = std::numeric_limits<int64_t>::min();

int g_checks = 0;
#define SN_CHECK(c)         \
    do {                    \
        CHECK(c);           \
        g_checks++;         \
    } while (0)

void CheckCreate(int64_t n) {
    const RefNum r(n);
    const CScriptNum s(n);
    SN_CHECK(Same(r, s));
    SN_CHECK(Same(RefNum(r.Int()), CScriptNum(s.getint())));
    if (s.getvch().size() <= CScriptNum::MAXIMUM_ELEMENT_SIZE) {
        // bytes -> number -> bytes, each side from the other side's encoding
        const CScriptNum s2(r.Bytes(), false);
        const RefNum r2 = RefNum::FromBytes(s.getvch());
        SN_CHECK(Same(r2, s2));
        SN_CHECK(CScriptNum(s.getvch(), true).getint64() == n); // the encoder is minimal
    } else {
        bool threw = false;
        try {
            CScriptNum(s.getvch(), false);
        } catch (const scriptnum_error&) {
            threw = true;
        }
        SN_CHECK(threw);
        threw = false;
        try {
            RefNum::FromBytes(r.Bytes());
        } catch (const scriptnum_error&) {
            threw = true;
        }
        SN_CHECK(threw);
    }
}

void CheckOps(int64_t a, int64_t b) {
    const RefNum ra(a), rb(b);
    const CScriptNum sa(a), sb(b);
    const bool addOk = !((b > 0 && a > I64MAX - b) || (b < 0 && a < I64MIN - b));
    if (addOk) {
        SN_CHECK(Same(RefNum(ra.v + rb.v), sa + sb));
        SN_CHECK(Same(RefNum(ra.v + rb.v), sa + b));
        SN_CHECK(Same(RefNum(ra.v + rb.v), sb + a));
    }
    if (!((b > 0 && a < I64MIN + b) || (b < 0 && a > I64MAX + b))) {
        SN_CHECK(Same(RefNum(ra.v - rb.v), sa - sb));
        SN_CHECK(Same(RefNum(ra.v - rb.v), sa - b));
    }
    if (!((a > 0 && b < I64MIN + a) || (a < 0 && b > I64MAX + a))) {
        SN_CHECK(Same(RefNum(rb.v - ra.v), sb - sa));
        SN_CHECK(Same(RefNum(rb.v - ra.v), sb - a));
    }
    if (a != I64MIN) SN_CHECK(Same(RefNum(-ra.v), -sa));
    // comparisons, against a number and against a plain int64
    SN_CHECK((ra.v == rb.v) == (sa == sb) && (ra.v == rb.v) == (sa == b));
    SN_CHECK((ra.v != rb.v) == (sa != sb) && (ra.v != rb.v) == (sa != b));
    SN_CHECK((ra.v < rb.v) == (sa < sb) && (ra.v < rb.v) == (sa < b));
    SN_CHECK((ra.v > rb.v) == (sa > sb) && (ra.v > rb.v) == (sa > b));
    SN_CHECK((ra.v <= rb.v) == (sa <= sb) && (ra.v <= rb.v) == (sa <= b));
    SN_CHECK((ra.v >= rb.v) == (sa >= sb) && (ra.v >= rb.v) == (sa >= b));
    SN_CHECK((sa == sa) && !(sa != sa) && !(sa < sa) && !(sa > sa) && (sa <= sa) && (sa >= sa));
}

} // namespace

TEST_CASE(scriptnum_tests, creation) {
    g_checks = 0;
    for (int64_t v : VALUES)
        for (int64_t o : OFFSETS) {
            CheckCreate(v);
            CheckCreate(v + o);
            CheckCreate(v - o);
        }
    CHECK(g_checks > 1000);
    // known encodings
    CHECK(CScriptNum(0).getvch().empty());
    CHECK(CScriptNum(-1).getvch() == std::vector<unsigned char>({0x81}));
    CHECK(CScriptNum(128).getvch() == std::vector<unsigned char>({0x80, 0x00}));
    CHECK(CScriptNum(-128).getvch() == std::vector<unsigned char>({0x80, 0x80}));
    CHECK(CScriptNum(255).getvch() == std::vector<unsigned char>({0xff, 0x00}));
    CHECK(CScriptNum(-0x7fffffffLL).getvch() == std::vector<unsigned char>({0xff, 0xff, 0xff, 0xff}));
    // negative zero and padded encodings are accepted unless minimality is required
    CHECK(CScriptNum(std::vector<unsigned char>({0x80}), false).getint64() == 0);
    CHECK(CScriptNum(std::vector<unsigned char>({0x01, 0x00}), false).getint64() == 1);
    bool threw = false;
    try {
        CScriptNum(std::vector<unsigned char>({0x01, 0x00}), true);
    } catch (const scriptnum_error&) {
        threw = true;
    }
    CHECK(threw);
}

TEST_CASE(scriptnum_tests, operators) {
    g_checks = 0;
    const size_t NV = sizeof(VALUES) / sizeof(VALUES[0]), NO = sizeof(OFFSETS) / sizeof(OFFSETS[0]);
    for (size_t i = 0; i < NV; i++)
        for (size_t j = 0; j < NO; j++) {
            const int64_t a = VALUES[i], b = VALUES[j % NV];
            CheckOps(a, a);
            CheckOps(a, -a);
            CheckOps(a, b);
            CheckOps(a, -b);
            CheckOps(a + b, b);
            CheckOps(a + b, -b);
            CheckOps(a - b, b);
            CheckOps(a - b, -b);
            CheckOps(a + b, a + b);
            CheckOps(a + b, a - b);
            CheckOps(a - b, a + b);
            CheckOps(a - b, a - b);
        }
    CHECK(g_checks > 10000);
}
