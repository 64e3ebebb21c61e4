// Fixed-width opaque blobs (uint160/uint256) and 256-bit unsigned arithmetic with
// the compact "nBits" encoding.
// Behaviour parity: reference src/uint256.h:19-150 (base_blob, GetHex reversed byte
// order) and src/arith_uint256.h:24-303 (SetCompact/GetCompact, operators).
#pragma once
#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace bcp {

template <unsigned BITS>
class base_blob {
public:
    static constexpr int WIDTH = BITS / 8;
    uint8_t data[WIDTH];

    base_blob() { memset(data, 0, sizeof(data)); }
    explicit base_blob(const std::vector<unsigned char>& v) {
        if (v.size() != sizeof(data)) throw std::invalid_argument("base_blob: bad vector size");
        memcpy(data, v.data(), sizeof(data));
    }
    bool IsNull() const {
        for (int i = 0; i < WIDTH; i++)
            if (data[i] != 0) return false;
        return true;
    }
    void SetNull() { memset(data, 0, sizeof(data)); }
    int Compare(const base_blob& o) const { return memcmp(data, o.data, sizeof(data)); }
    friend bool operator==(const base_blob& a, const base_blob& b) { return a.Compare(b) == 0; }
    friend bool operator!=(const base_blob& a, const base_blob& b) { return a.Compare(b) != 0; }
    friend bool operator<(const base_blob& a, const base_blob& b) { return a.Compare(b) < 0; }

    // Hex is printed most-significant byte first, i.e. data[] reversed (Bitcoin convention).
    std::string GetHex() const {
        static const char* hx = "0123456789abcdef";
        std::string s(WIDTH * 2, '0');
        for (int i = 0; i < WIDTH; i++) {
            uint8_t b = data[WIDTH - 1 - i];
            s[2 * i] = hx[b >> 4];
            s[2 * i + 1] = hx[b & 15];
        }
        return s;
    }
    void SetHex(const std::string& str) {
        memset(data, 0, sizeof(data));
        size_t p = 0;
        while (p < str.size() && isspace((unsigned char)str[p])) p++;
        if (str.size() - p >= 2 && str[p] == '0' && tolower(str[p + 1]) == 'x') p += 2;
        size_t end = p;
        while (end < str.size() && isxdigit((unsigned char)str[end])) end++;
        int idx = 0;
        auto hv = [](char c) -> int {
            if (c >= '0' && c <= '9') return c - '0';
            return (tolower(c) - 'a') + 10;
        };
        while (end > p && idx < WIDTH) {
            end--;
            uint8_t v = (uint8_t)hv(str[end]);
            if (end > p) {
                end--;
                v |= (uint8_t)(hv(str[end]) << 4);
            }
            data[idx++] = v;
        }
    }
    std::string ToString() const { return GetHex(); }
    unsigned char* begin() { return data; }
    unsigned char* end() { return data + WIDTH; }
    const unsigned char* begin() const { return data; }
    const unsigned char* end() const { return data + WIDTH; }
    static constexpr unsigned size() { return WIDTH; }
    uint64_t GetUint64(int pos) const {
        uint64_t v;
        memcpy(&v, data + pos * 8, 8);
        return v;
    }
    // Cheap hash for unordered containers (the data is already a hash).
    uint64_t GetCheapHash() const { return GetUint64(0); }

    template <typename Stream> void Serialize(Stream& s) const { s.write((const char*)data, sizeof(data)); }
    template <typename Stream> void Unserialize(Stream& s) { s.read((char*)data, sizeof(data)); }
};

class uint160 : public base_blob<160> {
public:
    uint160() {}
    explicit uint160(const std::vector<unsigned char>& v) : base_blob<160>(v) {}
};

class uint256 : public base_blob<256> {
public:
    uint256() {}
    uint256(const base_blob<256>& b) : base_blob<256>(b) {}
    explicit uint256(const std::vector<unsigned char>& v) : base_blob<256>(v) {}
    static uint256 FromHex(const std::string& s) { uint256 r; r.SetHex(s); return r; }
};

struct Uint256Hasher {
    size_t operator()(const uint256& h) const { return (size_t)h.GetCheapHash(); }
};

uint256 uint256S(const std::string& s);

class uint_error : public std::runtime_error {
public:
    explicit uint_error(const std::string& str) : std::runtime_error(str) {}
};

// 256-bit unsigned integer, 8 x 32-bit little-endian limbs.
class arith_uint256 {
public:
    static constexpr int WIDTH = 8;
    uint32_t pn[WIDTH];

    arith_uint256() { memset(pn, 0, sizeof(pn)); }
    arith_uint256(uint64_t b) {
        memset(pn, 0, sizeof(pn));
        pn[0] = (uint32_t)b;
        pn[1] = (uint32_t)(b >> 32);
    }
    explicit arith_uint256(const std::string& hex) { SetHex(hex); }

    arith_uint256 operator~() const { arith_uint256 r; for (int i = 0; i < WIDTH; i++) r.pn[i] = ~pn[i]; return r; }
    arith_uint256 operator-() const { arith_uint256 r = ~(*this); ++r; return r; }
    arith_uint256& operator^=(const arith_uint256& b) { for (int i = 0; i < WIDTH; i++) pn[i] ^= b.pn[i]; return *this; }
    arith_uint256& operator&=(const arith_uint256& b) { for (int i = 0; i < WIDTH; i++) pn[i] &= b.pn[i]; return *this; }
    arith_uint256& operator|=(const arith_uint256& b) { for (int i = 0; i < WIDTH; i++) pn[i] |= b.pn[i]; return *this; }
    arith_uint256& operator<<=(unsigned int shift);
    arith_uint256& operator>>=(unsigned int shift);
    arith_uint256& operator+=(const arith_uint256& b) {
        uint64_t carry = 0;
        for (int i = 0; i < WIDTH; i++) {
            uint64_t n = carry + pn[i] + b.pn[i];
            pn[i] = (uint32_t)n;
            carry = n >> 32;
        }
        return *this;
    }
    arith_uint256& operator-=(const arith_uint256& b) { *this += -b; return *this; }
    arith_uint256& operator+=(uint64_t b) { *this += arith_uint256(b); return *this; }
    arith_uint256& operator-=(uint64_t b) { *this += -arith_uint256(b); return *this; }
    arith_uint256& operator*=(uint32_t b32);
    arith_uint256& operator*=(const arith_uint256& b);
    arith_uint256& operator/=(const arith_uint256& b);
    arith_uint256& operator++() { int i = 0; while (i < WIDTH && ++pn[i] == 0) i++; return *this; }
    arith_uint256& operator--() { int i = 0; while (i < WIDTH && --pn[i] == (uint32_t)-1) i++; return *this; }

    int CompareTo(const arith_uint256& b) const {
        for (int i = WIDTH - 1; i >= 0; i--) {
            if (pn[i] < b.pn[i]) return -1;
            if (pn[i] > b.pn[i]) return 1;
        }
        return 0;
    }
    bool EqualTo(uint64_t b) const {
        for (int i = WIDTH - 1; i >= 2; i--) if (pn[i]) return false;
        return pn[1] == (uint32_t)(b >> 32) && pn[0] == (uint32_t)b;
    }
    friend arith_uint256 operator+(arith_uint256 a, const arith_uint256& b) { return a += b; }
    friend arith_uint256 operator-(arith_uint256 a, const arith_uint256& b) { return a -= b; }
    friend arith_uint256 operator*(arith_uint256 a, const arith_uint256& b) { return a *= b; }
    friend arith_uint256 operator/(arith_uint256 a, const arith_uint256& b) { return a /= b; }
    friend arith_uint256 operator*(arith_uint256 a, uint32_t b) { return a *= b; }
    friend arith_uint256 operator|(arith_uint256 a, const arith_uint256& b) { return a |= b; }
    friend arith_uint256 operator&(arith_uint256 a, const arith_uint256& b) { return a &= b; }
    friend arith_uint256 operator^(arith_uint256 a, const arith_uint256& b) { return a ^= b; }
    friend arith_uint256 operator>>(arith_uint256 a, int s) { return a >>= s; }
    friend arith_uint256 operator<<(arith_uint256 a, int s) { return a <<= s; }
    friend bool operator==(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) == 0; }
    friend bool operator!=(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) != 0; }
    friend bool operator>(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) > 0; }
    friend bool operator<(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) < 0; }
    friend bool operator>=(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) >= 0; }
    friend bool operator<=(const arith_uint256& a, const arith_uint256& b) { return a.CompareTo(b) <= 0; }
    friend bool operator==(const arith_uint256& a, uint64_t b) { return a.EqualTo(b); }
    friend bool operator!=(const arith_uint256& a, uint64_t b) { return !a.EqualTo(b); }

    unsigned int bits() const;
    uint64_t GetLow64() const { return pn[0] | ((uint64_t)pn[1] << 32); }
    double getdouble() const;
    std::string GetHex() const;
    void SetHex(const std::string& s);
    std::string ToString() const { return GetHex(); }

    // Compact nBits encoding (reference src/arith_uint256.cpp SetCompact/GetCompact).
    arith_uint256& SetCompact(uint32_t nCompact, bool* pfNegative = nullptr, bool* pfOverflow = nullptr);
    uint32_t GetCompact(bool fNegative = false) const;
};

uint256 ArithToUint256(const arith_uint256& a);
arith_uint256 UintToArith256(const uint256& a);

} // namespace bcp
