// Command-line arguments, string/number parsing and formatting, the peer-time median filter.
// Parity: reference src/test/getarg_tests.cpp (boolarg, stringarg, intarg, doubledash,
// boolargno), src/test/util_tests.cpp (ParseHex/HexStr, ParseParameters/GetArg, FormatMoney/
// ParseMoney, IsHex, strprintf numbers, ParseInt32/64, ParseUInt32, ParseDouble,
// FormatSubVersion, ParseFixedPoint) and src/test/timedata_tests.cpp (util_MedianFilter).
// Money and fixed-point cases are generated over every power of ten instead of listed.
#include "test/unittest.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <cmath>
#include <limits>

namespace bcp {
namespace {

// a fresh ArgsManager parsed from a space-separated command line
struct Args {
    ArgsManager am;
    explicit Args(const std::string& line) {
        std::vector<std::string> words{"bcpd"};
        for (const std::string& w : SplitString(line, ' '))
            if (!w.empty()) words.push_back(w);
        std::vector<const char*> argv;
        for (const std::string& w : words) argv.push_back(w.c_str());
        am.ParseParameters((int)argv.size(), argv.data());
    }
};

} // namespace

TEST_CASE(getarg_tests, boolean_options) {
    // (command line, value of -opt with default false, with default true)
    struct Row {
        const char* line;
        bool whenFalse, whenTrue;
    } rows[] = {
        {"", false, true},
        {"-opt", true, true},
        {"-opt=", true, true},
        {"-opt=1", true, true},
        {"-opt=0", false, false},
        {"-noopt", false, false},
        {"-noopt=1", false, false},
        {"-noopt=0", true, true},
        {"-opt -noopt", false, false},     // the later one wins
        {"-noopt -opt", true, true},
        {"-opt=1 -noopt=1", false, false},
        {"-opt=0 -noopt=0", true, true},
        {"--opt=1", true, true},           // a double dash reads as one
        {"--noopt=1", false, false},
        {"-opt --noopt", false, false},
        {"-optx", false, true},            // other names do not match
        {"-op", false, true},
    };
    for (const Row& r : rows) {
        Args a(r.line);
        CHECK_EQ(a.am.GetBoolArg("-opt", false), r.whenFalse);
        CHECK_EQ(a.am.GetBoolArg("-opt", true), r.whenTrue);
    }
}

TEST_CASE(getarg_tests, string_and_integer_options) {
    CHECK_EQ(Args("").am.GetArg("-name", "dflt"), std::string("dflt"));
    CHECK_EQ(Args("-name -other").am.GetArg("-name", "dflt"), std::string(""));
    CHECK_EQ(Args("-name=").am.GetArg("-name", "dflt"), std::string(""));
    CHECK_EQ(Args("-name=42").am.GetArg("-name", "dflt"), std::string("42"));
    CHECK_EQ(Args("-name=forty-two").am.GetArg("-name", ""), std::string("forty-two"));
    CHECK_EQ(Args("--name=verbose --level=3").am.GetArg("-name", ""), std::string("verbose"));
    CHECK_EQ(Args("--name=verbose --level=3").am.GetArg("-level", (int64_t)0), (int64_t)3);
    CHECK_EQ(Args("").am.GetArg("-n", (int64_t)42), (int64_t)42);
    CHECK_EQ(Args("-n -m").am.GetArg("-n", (int64_t)42), (int64_t)0); // present without a value
    CHECK_EQ(Args("-n=7 -m=8").am.GetArg("-m", (int64_t)0), (int64_t)8);
    CHECK_EQ(Args("-n=abc").am.GetArg("-n", (int64_t)42), (int64_t)0); // unparsable reads as 0
    CHECK_EQ(Args("-n=-12").am.GetArg("-n", (int64_t)0), (int64_t)-12);
    // repeated options keep every value, GetArg reads the last
    Args rep("-connect=a -connect=b -connect=c");
    CHECK_EQ(rep.am.GetArgs("-connect").size(), (size_t)3);
    CHECK_EQ(rep.am.GetArg("-connect", ""), std::string("c"));
    CHECK(rep.am.IsArgSet("-connect"));
    CHECK(!rep.am.IsArgSet("-bind"));
    // arguments stop at the first word that is not an option
    Args pos("-a=1 getblock -b=2");
    CHECK(pos.am.IsArgSet("-a"));
    CHECK(!pos.am.IsArgSet("-b"));
}

TEST_CASE(getarg_tests, soft_and_forced) {
    Args a("-set=1");
    CHECK(!a.am.SoftSetArg("-set", "2"));
    CHECK_EQ(a.am.GetArg("-set", ""), std::string("1"));
    CHECK(a.am.SoftSetArg("-unset", "v"));
    CHECK_EQ(a.am.GetArg("-unset", ""), std::string("v"));
    CHECK(a.am.SoftSetBoolArg("-flag", false));
    CHECK(!a.am.GetBoolArg("-flag", true));
    a.am.ForceSetArg("-set", "9");
    CHECK_EQ(a.am.GetArg("-set", (int64_t)0), (int64_t)9);
    a.am.ClearArg("-set");
    CHECK(!a.am.IsArgSet("-set"));
}

TEST_CASE(util_tests, hex) {
    // every byte value round-trips; upper and lower case parse alike
    std::vector<unsigned char> all(256);
    for (int i = 0; i < 256; i++) all[i] = (unsigned char)i;
    const std::string h = HexStr(all);
    CHECK_EQ(h.size(), (size_t)512);
    CHECK(ParseHex(h) == all);
    CHECK(ParseHex(ToUpper(h)) == all);
    CHECK_EQ(HexStr(ParseHex("00ff10")), std::string("00ff10"));
    // whitespace between bytes is skipped, parsing stops at the first non-hex character
    CHECK(ParseHex(" 12 34 56 ") == (std::vector<unsigned char>{0x12, 0x34, 0x56}));
    CHECK(ParseHex("1234zz56") == (std::vector<unsigned char>{0x12, 0x34}));
    CHECK(ParseHex("").empty());
    CHECK(IsHex("00"));
    CHECK(IsHex("abcDEF0123456789"));
    CHECK(!IsHex(""));
    CHECK(!IsHex("0"));     // odd length
    CHECK(!IsHex("0x00"));
    CHECK(!IsHex("ag"));
    CHECK(!IsHex(" 00"));
}

TEST_CASE(util_tests, money) {
    // FormatMoney prints at least two decimals and no trailing zeros beyond them
    CHECK_EQ(FormatMoney(0), std::string("0.00"));
    CHECK_EQ(FormatMoney(-COIN), std::string("-1.00"));
    CHECK_EQ(FormatMoney(1234567891LL), std::string("12.34567891"));
    int64_t unit = COIN;
    for (int e = 0; e <= 8; e++) { // 10^8 BCP .. 1 BCP
        const int64_t v = unit * (int64_t)std::pow(10, e);
        std::string want = "1" + std::string(e, '0') + ".00";
        CHECK_EQ(FormatMoney(v), want);
        int64_t back = -1;
        CHECK(ParseMoney(want, back));
        CHECK_EQ(back, v);
    }
    for (int e = 1; e <= 8; e++) { // 0.1 .. 0.00000001
        const int64_t v = COIN / (int64_t)std::pow(10, e);
        std::string want = "0." + std::string(e - 1, '0') + "1";
        if (want.size() < 4) want += "0";
        CHECK_EQ(FormatMoney(v), want);
        int64_t back = -1;
        CHECK(ParseMoney(want, back));
        CHECK_EQ(back, v);
    }
    int64_t r = 0;
    CHECK(ParseMoney("7", r));
    CHECK_EQ(r, 7 * COIN);
    CHECK(ParseMoney(" 3.5 ", r));
    CHECK_EQ(r, 350000000LL);
    CHECK(!ParseMoney("92233720368.54775808", r)); // beyond 63 bits
    CHECK(!ParseMoney("-2", r));
    CHECK(!ParseMoney("1.000000001", r));           // finer than a satoshi
    CHECK(!ParseMoney("1e5", r));
    CHECK(ParseMoney("", r) && r == 0); // as in the reference, nothing reads as zero
    CHECK(!ParseMoney("12345678901", r)); // eleven integer digits
}

TEST_CASE(util_tests, integers) {
    int32_t i32 = 0;
    CHECK(ParseInt32("0", &i32) && i32 == 0);
    CHECK(ParseInt32("-2147483648", &i32) && i32 == std::numeric_limits<int32_t>::min());
    CHECK(ParseInt32("2147483647", &i32) && i32 == std::numeric_limits<int32_t>::max());
    CHECK(ParseInt32("+77", &i32) && i32 == 77);
    CHECK(ParseInt32("00042", &i32) && i32 == 42); // leading zeros are decimal, not octal
    for (const char* bad : {"2147483648", "-2147483649", "", " 1", "1 ", "1a", "0x10", "--1", "1.0", "N/A"})
        CHECK(!ParseInt32(bad, &i32));
    int64_t i64 = 0;
    CHECK(ParseInt64("9223372036854775807", &i64) && i64 == std::numeric_limits<int64_t>::max());
    CHECK(ParseInt64("-9223372036854775808", &i64) && i64 == std::numeric_limits<int64_t>::min());
    CHECK(ParseInt64("-1234567890123", &i64) && i64 == -1234567890123LL);
    for (const char* bad : {"9223372036854775808", "-9223372036854775809", "", "12 ", "1e3", "0x1"})
        CHECK(!ParseInt64(bad, &i64));
    uint32_t u32 = 0;
    CHECK(ParseUInt32("4294967295", &u32) && u32 == 4294967295u);
    CHECK(ParseUInt32("+9", &u32) && u32 == 9);
    for (const char* bad : {"4294967296", "-1", "-0", "", " 5", "5x"}) CHECK(!ParseUInt32(bad, &u32));
    double d = 0;
    CHECK(ParseDouble("1.5", &d) && d == 1.5);
    CHECK(ParseDouble("-1e3", &d) && d == -1000.0);
    CHECK(ParseDouble("0", &d) && d == 0.0);
    for (const char* bad : {"", "1.0x", "0x10", "nan?", " 1"}) CHECK(!ParseDouble(bad, &d));
}

TEST_CASE(util_tests, fixed_point) {
    int64_t v = 0;
    // k * 10^-e for every scale the 8-decimal parser accepts
    for (int e = 0; e <= 8; e++) {
        const std::string s = e == 0 ? "3" : "0." + std::string(e - 1, '0') + "3";
        CHECK(ParseFixedPoint(s, 8, &v));
        CHECK_EQ(v, 3 * (int64_t)std::pow(10, 8 - e));
        CHECK(ParseFixedPoint("-" + s, 8, &v));
        CHECK_EQ(v, -3 * (int64_t)std::pow(10, 8 - e));
    }
    CHECK(ParseFixedPoint("2.5e2", 8, &v) && v == 25000000000LL);
    CHECK(ParseFixedPoint("2.5e-2", 8, &v) && v == 2500000LL);
    CHECK(ParseFixedPoint("1.50000000000000000000", 8, &v) && v == 150000000LL);
    CHECK(ParseFixedPoint("9999999999.99999999", 8, &v) && v == 999999999999999999LL);
    CHECK(ParseFixedPoint("-9999999999.99999999", 8, &v) && v == -999999999999999999LL);
    for (const char* bad : {"", "-", ".5", "00.5", "-05", "5.", "1..0", "1e", "1e-", "x1", "1x", "0.000000001",
                            "10000000000", "1e10", "1.0e-9", "1 "})
        CHECK(!ParseFixedPoint(bad, 8, &v));
}

TEST_CASE(util_tests, formatting) {
    CHECK_EQ(strprintf("%d %u %s", -7, 7u, "x"), std::string("-7 7 x"));
    CHECK_EQ(strprintf("%lld", (long long)std::numeric_limits<int64_t>::min()), std::string("-9223372036854775808"));
    CHECK_EQ(strprintf("%llu", (unsigned long long)std::numeric_limits<uint64_t>::max()),
             std::string("18446744073709551615"));
    CHECK_EQ(strprintf("%08x", 0xbeefu), std::string("0000beef"));
    CHECK_EQ(strprintf("%.3f", 2.0 / 3), std::string("0.667"));
    CHECK_EQ(strprintf("%s", std::string(5000, 'z').c_str()).size(), (size_t)5000); // longer than any fixed buffer
    CHECK_EQ(FormatSubVersion("Name", 170000, {}), std::string("/Name:0.17.0/"));
    CHECK_EQ(FormatSubVersion("Name", 170000, {"c1"}), std::string("/Name:0.17.0(c1)/"));
    CHECK_EQ(FormatSubVersion("Name", 170100, {"c1", "c2"}), std::string("/Name:0.17.1(c1; c2)/"));
    CHECK_EQ(SanitizeString("a<b>c\x01"), std::string("abc"));
    CHECK_EQ(TrimString("  \tx y \n"), std::string("x y"));
}

TEST_CASE(timedata_tests, median_filter) {
    MedianFilter<int> f(5, 15);
    CHECK_EQ(f.median(), 15);
    f.input(20); // 15 20
    CHECK_EQ(f.median(), 17);
    f.input(30); // 15 20 30
    CHECK_EQ(f.median(), 20);
    f.input(3); // 3 15 20 30
    CHECK_EQ(f.median(), 17);
    f.input(7); // 3 7 15 20 30
    CHECK_EQ(f.median(), 15);
    f.input(18); // the oldest (15) leaves: 3 7 18 20 30
    CHECK_EQ(f.median(), 18);
    f.input(0); // 20 leaves: 0 3 7 18 30
    CHECK_EQ(f.median(), 7);
    CHECK_EQ(f.size(), 5);
    // against a brute-force median over a random stream
    MedianFilter<int64_t> g(7, 0);
    std::vector<int64_t> window{0};
    uint64_t x = 88172645463325252ULL;
    for (int i = 0; i < 2000; i++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        const int64_t v = (int64_t)(x % 2001) - 1000;
        g.input(v);
        window.push_back(v);
        if (window.size() > 7) window.erase(window.begin());
        std::vector<int64_t> s = window;
        std::sort(s.begin(), s.end());
        const int64_t want = s.size() & 1 ? s[s.size() / 2] : (s[s.size() / 2 - 1] + s[s.size() / 2]) / 2;
        CHECK_EQ(g.median(), want);
    }
}

} // namespace bcp
