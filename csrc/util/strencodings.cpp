#include "util/strencodings.h"

#include <cerrno>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>

namespace bcp {

static int HexDigit(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

bool IsHex(const std::string& str) {
    for (char c : str)
        if (HexDigit(c) < 0) return false;
    return !str.empty() && str.size() % 2 == 0;
}

bool IsHexNumber(const std::string& str) {
    size_t start = 0;
    if (str.size() > 2 && str[0] == '0' && str[1] == 'x') start = 2;
    for (size_t i = start; i < str.size(); ++i)
        if (HexDigit(str[i]) < 0) return false;
    return str.size() > start;
}

std::vector<unsigned char> ParseHex(const std::string& str) {
    std::vector<unsigned char> out;
    size_t i = 0;
    while (true) {
        while (i < str.size() && isspace((unsigned char)str[i])) i++;
        if (i >= str.size()) break;
        int hi = HexDigit(str[i]);
        if (hi < 0 || i + 1 >= str.size()) break;
        int lo = HexDigit(str[i + 1]);
        if (lo < 0) break;
        out.push_back((unsigned char)((hi << 4) | lo));
        i += 2;
    }
    return out;
}

std::string HexStr(const unsigned char* b, const unsigned char* e) {
    static const char* hx = "0123456789abcdef";
    std::string s;
    s.reserve((e - b) * 2);
    for (; b < e; ++b) {
        s.push_back(hx[*b >> 4]);
        s.push_back(hx[*b & 15]);
    }
    return s;
}

std::string EncodeBase64(const unsigned char* p, size_t n) {
    static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    std::string out;
    size_t i = 0;
    for (; i + 2 < n; i += 3) {
        uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
        out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += tbl[(v >> 6) & 63]; out += tbl[v & 63];
    }
    if (i + 1 == n) {
        uint32_t v = p[i] << 16;
        out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += "==";
    } else if (i + 2 == n) {
        uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
        out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += tbl[(v >> 6) & 63]; out += '=';
    }
    return out;
}
std::string EncodeBase64(const std::string& s) { return EncodeBase64((const unsigned char*)s.data(), s.size()); }

std::vector<unsigned char> DecodeBase64(const std::string& s, bool* invalid) {
    auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z') return c - 'A';
        if (c >= 'a' && c <= 'z') return c - 'a' + 26;
        if (c >= '0' && c <= '9') return c - '0' + 52;
        if (c == '+') return 62;
        if (c == '/') return 63;
        return -1;
    };
    std::vector<unsigned char> out;
    uint32_t acc = 0;
    int bits = 0;
    size_t i = 0;
    bool bad = false;
    for (; i < s.size(); ++i) {
        int v = val(s[i]);
        if (v < 0) break;
        acc = (acc << 6) | v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back((unsigned char)(acc >> bits));
        }
    }
    size_t pads = 0;
    while (i < s.size() && s[i] == '=') { ++i; ++pads; }
    if (i != s.size()) bad = true;
    if ((s.size() % 4) != 0) bad = true;
    if (invalid) *invalid = bad;
    return out;
}

std::string EncodeBase32(const unsigned char* p, size_t n) {
    static const char* tbl = "abcdefghijklmnopqrstuvwxyz234567";
    std::string out;
    uint64_t acc = 0;
    int bits = 0;
    for (size_t i = 0; i < n; ++i) {
        acc = (acc << 8) | p[i];
        bits += 8;
        while (bits >= 5) { bits -= 5; out += tbl[(acc >> bits) & 31]; }
    }
    if (bits > 0) out += tbl[(acc << (5 - bits)) & 31];
    while (out.size() % 8) out += '=';
    return out;
}

std::vector<unsigned char> DecodeBase32(const std::string& s, bool* invalid) {
    std::vector<unsigned char> out;
    uint64_t acc = 0;
    int bits = 0;
    size_t i = 0;
    for (; i < s.size(); ++i) {
        char c = s[i];
        int v;
        if (c >= 'a' && c <= 'z') v = c - 'a';
        else if (c >= 'A' && c <= 'Z') v = c - 'A';
        else if (c >= '2' && c <= '7') v = c - '2' + 26;
        else break;
        acc = (acc << 5) | v;
        bits += 5;
        if (bits >= 8) { bits -= 8; out.push_back((unsigned char)(acc >> bits)); }
    }
    while (i < s.size() && s[i] == '=') ++i;
    if (invalid) *invalid = i != s.size() || s.size() % 8;
    return out;
}

static bool ParsePrechecks(const std::string& str) {
    if (str.empty()) return false;
    if (isspace((unsigned char)str[0]) || isspace((unsigned char)str[str.size() - 1])) return false;
    if (str.size() != strlen(str.c_str())) return false;
    return true;
}

bool ParseInt32(const std::string& str, int32_t* out) {
    if (!ParsePrechecks(str)) return false;
    char* endp = nullptr;
    errno = 0;
    long n = strtol(str.c_str(), &endp, 10);
    if (out) *out = (int32_t)n;
    return endp && *endp == 0 && !errno && n >= std::numeric_limits<int32_t>::min() &&
           n <= std::numeric_limits<int32_t>::max();
}

bool ParseInt64(const std::string& str, int64_t* out) {
    if (!ParsePrechecks(str)) return false;
    char* endp = nullptr;
    errno = 0;
    long long n = strtoll(str.c_str(), &endp, 10);
    if (out) *out = (int64_t)n;
    return endp && *endp == 0 && !errno;
}

bool ParseUInt32(const std::string& str, uint32_t* out) {
    if (!ParsePrechecks(str)) return false;
    if (str[0] == '-') return false;
    char* endp = nullptr;
    errno = 0;
    unsigned long long n = strtoull(str.c_str(), &endp, 10);
    if (out) *out = (uint32_t)n;
    return endp && *endp == 0 && !errno && n <= std::numeric_limits<uint32_t>::max();
}

bool ParseDouble(const std::string& str, double* out) {
    if (!ParsePrechecks(str)) return false;
    if (str.size() >= 2 && str[0] == '0' && str[1] == 'x') return false;
    char* endp = nullptr;
    errno = 0;
    double d = strtod(str.c_str(), &endp);
    if (out) *out = d;
    return endp && *endp == 0 && !errno;
}

int64_t atoi64(const std::string& s) { return strtoll(s.c_str(), nullptr, 10); }

// Parse "123.456e-2"-style fixed point (reference ParseFixedPoint).
bool ParseFixedPoint(const std::string& val, int decimals, int64_t* amount_out) {
    const int64_t UPPER = 1000000000000000000LL - 1;
    int64_t mantissa = 0, exponent = 0;
    int mantissa_tzeros = 0;
    bool mantissa_sign = false, exponent_sign = false;
    int ptr = 0, end = (int)val.size(), point_ofs = 0;
    auto process = [&](char ch) -> bool {
        if (ch == '0') ++mantissa_tzeros;
        else {
            for (int i = 0; i <= mantissa_tzeros; ++i) {
                if (mantissa > (UPPER / 10LL)) return false;
                mantissa *= 10;
            }
            mantissa += ch - '0';
            mantissa_tzeros = 0;
        }
        return true;
    };
    if (ptr < end && val[ptr] == '-') { mantissa_sign = true; ++ptr; }
    if (ptr < end) {
        if (val[ptr] == '0') ++ptr;
        else if (val[ptr] >= '1' && val[ptr] <= '9') {
            while (ptr < end && isdigit((unsigned char)val[ptr])) {
                if (!process(val[ptr])) return false;
                ++ptr;
            }
        } else return false;
    } else return false;
    if (ptr < end && val[ptr] == '.') {
        ++ptr;
        if (ptr < end && isdigit((unsigned char)val[ptr])) {
            while (ptr < end && isdigit((unsigned char)val[ptr])) {
                if (!process(val[ptr])) return false;
                ++ptr;
                ++point_ofs;
            }
        } else return false;
    }
    if (ptr < end && (val[ptr] == 'e' || val[ptr] == 'E')) {
        ++ptr;
        if (ptr < end && val[ptr] == '+') ++ptr;
        else if (ptr < end && val[ptr] == '-') { exponent_sign = true; ++ptr; }
        if (ptr < end && isdigit((unsigned char)val[ptr])) {
            while (ptr < end && isdigit((unsigned char)val[ptr])) {
                if (exponent > (UPPER / 10LL)) return false;
                exponent = exponent * 10 + val[ptr] - '0';
                ++ptr;
            }
        } else return false;
    }
    if (ptr != end) return false;
    if (exponent_sign) exponent = -exponent;
    exponent = exponent - point_ofs + mantissa_tzeros;
    if (mantissa_sign) mantissa = -mantissa;
    exponent += decimals;
    if (exponent < 0) return false;
    if (exponent >= 18) return false;
    for (int i = 0; i < exponent; ++i) {
        if (mantissa > (UPPER / 10LL) || mantissa < -(UPPER / 10LL)) return false;
        mantissa *= 10;
    }
    if (mantissa > UPPER || mantissa < -UPPER) return false;
    if (amount_out) *amount_out = mantissa;
    return true;
}

std::string FormatMoney(int64_t n) {
    int64_t n_abs = n > 0 ? n : -n;
    int64_t quotient = n_abs / 100000000;
    int64_t remainder = n_abs % 100000000;
    char buf[64];
    snprintf(buf, sizeof(buf), "%lld.%08lld", (long long)quotient, (long long)remainder);
    std::string str(buf);
    int nTrim = 0;
    for (int i = (int)str.size() - 1; str[i] == '0' && isdigit((unsigned char)str[i - 2]); --i) ++nTrim;
    if (nTrim) str.erase(str.size() - nTrim, nTrim);
    if (n < 0) str.insert((unsigned int)0, 1, '-');
    return str;
}

// Reference utilmoneystr.cpp ParseMoney: optional surrounding whitespace, at most ten integer
// digits, at most eight decimals, no sign or exponent ("" reads as zero).
bool ParseMoney(const std::string& s, int64_t& n) {
    size_t i = 0;
    while (i < s.size() && isspace((unsigned char)s[i])) i++;
    int64_t whole = 0, units = 0;
    int wholeDigits = 0;
    for (; i < s.size() && isdigit((unsigned char)s[i]); i++, wholeDigits++)
        if (wholeDigits < 11) whole = whole * 10 + (s[i] - '0');
    if (i < s.size() && s[i] == '.') {
        i++;
        int64_t mult = 10000000; // 0.1 BCP in satoshis
        for (; i < s.size() && isdigit((unsigned char)s[i]) && mult > 0; i++, mult /= 10) units += mult * (s[i] - '0');
    }
    for (; i < s.size(); i++)
        if (!isspace((unsigned char)s[i])) return false;
    if (wholeDigits > 10) return false; // 63-bit overflow guard
    n = whole * 100000000 + units;
    return true;
}

std::string SanitizeString(const std::string& str) {
    static const std::string ok = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz01234567890 .,;-_/:?@()";
    std::string r;
    for (char c : str)
        if (ok.find(c) != std::string::npos) r.push_back(c);
    return r;
}

std::string ToLower(std::string s) { for (auto& c : s) c = (char)tolower((unsigned char)c); return s; }
std::string ToUpper(std::string s) { for (auto& c : s) c = (char)toupper((unsigned char)c); return s; }

std::vector<std::string> SplitString(const std::string& s, char sep) {
    std::vector<std::string> out;
    std::string cur;
    for (char c : s) {
        if (c == sep) { out.push_back(cur); cur.clear(); }
        else cur.push_back(c);
    }
    out.push_back(cur);
    return out;
}

std::string TrimString(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && isspace((unsigned char)s[b])) ++b;
    while (e > b && isspace((unsigned char)s[e - 1])) --e;
    return s.substr(b, e - b);
}

std::string strprintf(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char buf[512];
    va_list ap2;
    va_copy(ap2, ap);
    int n = vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (n < (int)sizeof(buf)) { va_end(ap2); return std::string(buf, n > 0 ? n : 0); }
    std::string s(n + 1, '\0');
    vsnprintf(&s[0], n + 1, fmt, ap2);
    va_end(ap2);
    s.resize(n);
    return s;
}

} // namespace bcp
