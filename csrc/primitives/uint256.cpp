#include "primitives/uint256.h"
#include "crypto/common.h"

namespace bcp {

uint256 uint256S(const std::string& s) { uint256 r; r.SetHex(s); return r; }

arith_uint256& arith_uint256::operator<<=(unsigned int shift) {
    arith_uint256 a(*this);
    memset(pn, 0, sizeof(pn));
    int k = shift / 32;
    shift = shift % 32;
    for (int i = 0; i < WIDTH; i++) {
        if (i + k + 1 < WIDTH && shift != 0) pn[i + k + 1] |= (a.pn[i] >> (32 - shift));
        if (i + k < WIDTH) pn[i + k] |= (a.pn[i] << shift);
    }
    return *this;
}

arith_uint256& arith_uint256::operator>>=(unsigned int shift) {
    arith_uint256 a(*this);
    memset(pn, 0, sizeof(pn));
    int k = shift / 32;
    shift = shift % 32;
    for (int i = 0; i < WIDTH; i++) {
        if (i - k - 1 >= 0 && shift != 0) pn[i - k - 1] |= (a.pn[i] << (32 - shift));
        if (i - k >= 0) pn[i - k] |= (a.pn[i] >> shift);
    }
    return *this;
}

arith_uint256& arith_uint256::operator*=(uint32_t b32) {
    uint64_t carry = 0;
    for (int i = 0; i < WIDTH; i++) {
        uint64_t n = carry + (uint64_t)b32 * pn[i];
        pn[i] = (uint32_t)n;
        carry = n >> 32;
    }
    return *this;
}

arith_uint256& arith_uint256::operator*=(const arith_uint256& b) {
    arith_uint256 a;
    for (int j = 0; j < WIDTH; j++) {
        uint64_t carry = 0;
        for (int i = 0; i + j < WIDTH; i++) {
            uint64_t n = carry + a.pn[i + j] + (uint64_t)pn[j] * b.pn[i];
            a.pn[i + j] = (uint32_t)n;
            carry = n >> 32;
        }
    }
    *this = a;
    return *this;
}

unsigned int arith_uint256::bits() const {
    for (int pos = WIDTH - 1; pos >= 0; pos--) {
        if (pn[pos]) {
            for (int nbits = 31; nbits > 0; nbits--)
                if (pn[pos] & (1U << nbits)) return 32 * pos + nbits + 1;
            return 32 * pos + 1;
        }
    }
    return 0;
}

arith_uint256& arith_uint256::operator/=(const arith_uint256& b) {
    arith_uint256 div = b;
    arith_uint256 num = *this;
    memset(pn, 0, sizeof(pn));
    int num_bits = num.bits();
    int div_bits = div.bits();
    if (div_bits == 0) throw uint_error("Division by zero");
    if (div_bits > num_bits) return *this;
    int shift = num_bits - div_bits;
    div <<= shift;
    while (shift >= 0) {
        if (num >= div) {
            num -= div;
            pn[shift / 32] |= (1U << (shift & 31));
        }
        div >>= 1;
        shift--;
    }
    return *this;
}

double arith_uint256::getdouble() const {
    double ret = 0.0, fact = 1.0;
    for (int i = 0; i < WIDTH; i++) {
        ret += fact * pn[i];
        fact *= 4294967296.0;
    }
    return ret;
}

std::string arith_uint256::GetHex() const { return ArithToUint256(*this).GetHex(); }
void arith_uint256::SetHex(const std::string& s) { *this = UintToArith256(uint256S(s)); }

arith_uint256& arith_uint256::SetCompact(uint32_t nCompact, bool* pfNegative, bool* pfOverflow) {
    int nSize = nCompact >> 24;
    uint32_t nWord = nCompact & 0x007fffff;
    if (nSize <= 3) {
        nWord >>= 8 * (3 - nSize);
        *this = nWord;
    } else {
        *this = nWord;
        *this <<= 8 * (nSize - 3);
    }
    if (pfNegative) *pfNegative = nWord != 0 && (nCompact & 0x00800000) != 0;
    if (pfOverflow)
        *pfOverflow = nWord != 0 && ((nSize > 34) || (nWord > 0xff && nSize > 33) || (nWord > 0xffff && nSize > 32));
    return *this;
}

uint32_t arith_uint256::GetCompact(bool fNegative) const {
    int nSize = (bits() + 7) / 8;
    uint32_t nCompact = 0;
    if (nSize <= 3) {
        nCompact = (uint32_t)(GetLow64() << 8 * (3 - nSize));
    } else {
        arith_uint256 bn = *this >> 8 * (nSize - 3);
        nCompact = (uint32_t)bn.GetLow64();
    }
    // The 0x00800000 bit denotes the sign; if it is already set, divide the mantissa by 256.
    if (nCompact & 0x00800000) {
        nCompact >>= 8;
        nSize++;
    }
    nCompact |= nSize << 24;
    nCompact |= (fNegative && (nCompact & 0x007fffff) ? 0x00800000 : 0);
    return nCompact;
}

uint256 ArithToUint256(const arith_uint256& a) {
    uint256 b;
    for (int x = 0; x < arith_uint256::WIDTH; ++x) WriteLE32(b.begin() + x * 4, a.pn[x]);
    return b;
}

arith_uint256 UintToArith256(const uint256& a) {
    arith_uint256 b;
    for (int x = 0; x < arith_uint256::WIDTH; ++x) b.pn[x] = ReadLE32(a.begin() + x * 4);
    return b;
}

} // namespace bcp
