// Equihash CPU reference. See equihash.h for the parity map.
#include "consensus/equihash.h"
#include "crypto/common.h"

#include <algorithm>
#include <cassert>
#include <cstring>
#include <stdexcept>

namespace bcp {

bool EquihashParams::Valid() const {
    if (K == 0 || K >= N || N % 8 != 0) return false;
    if (N > 512) return false;
    if ((N / (K + 1)) + 1 >= 32) return false;
    if (N % (K + 1) != 0) return false;
    return true;
}

std::string EquihashParams::ToString() const { return "Equihash(" + std::to_string(N) + "," + std::to_string(K) + ")"; }

bool EquihashParamsSupported(unsigned n, unsigned k) {
    return (n == 200 && k == 9) || (n == 96 && k == 5) || (n == 96 && k == 3) || (n == 48 && k == 5);
}

CBlake2b EhInitialiseState(const EquihashParams& p) {
    unsigned char personal[16] = {0};
    memcpy(personal, "ZcashPoW", 8);
    WriteLE32(personal + 8, p.N);
    WriteLE32(personal + 12, p.K);
    return CBlake2b((512 / p.N) * p.N / 8, nullptr, 0, nullptr, personal);
}

void EhGenerateHash(const CBlake2b& base, uint32_t g, unsigned char* out) {
    CBlake2b st = base;
    unsigned char le[4];
    WriteLE32(le, g);
    st.Write(le, 4);
    st.Finalize(out);
}

// Reads `bit_len`-bit big-endian groups from `in` and writes each group as a
// big-endian integer in ceil(bit_len/8)+byte_pad bytes (leading pad bytes zero).
void ExpandArray(const unsigned char* in, size_t in_len, unsigned char* out, size_t out_len,
                 size_t bit_len, size_t byte_pad) {
    if (bit_len < 8 || bit_len + 7 > 32) throw std::invalid_argument("ExpandArray bit_len");
    const size_t out_width = (bit_len + 7) / 8 + byte_pad;
    const size_t groups = 8 * in_len / bit_len;
    if (out_len != groups * out_width) throw std::invalid_argument("ExpandArray out_len");
    const uint32_t mask = (bit_len == 32) ? 0xffffffffu : ((1u << bit_len) - 1);
    uint64_t acc = 0;
    size_t acc_bits = 0, pos = 0;
    for (size_t g = 0; g < groups; ++g) {
        while (acc_bits < bit_len) {
            acc = (acc << 8) | in[pos++];
            acc_bits += 8;
        }
        uint32_t v = (uint32_t)(acc >> (acc_bits - bit_len)) & mask;
        acc_bits -= bit_len;
        unsigned char* o = out + g * out_width;
        memset(o, 0, byte_pad);
        const size_t vb = out_width - byte_pad;
        for (size_t b = 0; b < vb; ++b) o[byte_pad + b] = (unsigned char)(v >> (8 * (vb - 1 - b)));
    }
}

void CompressArray(const unsigned char* in, size_t in_len, unsigned char* out, size_t out_len,
                   size_t bit_len, size_t byte_pad) {
    if (bit_len < 8 || bit_len + 7 > 32) throw std::invalid_argument("CompressArray bit_len");
    const size_t in_width = (bit_len + 7) / 8 + byte_pad;
    if (out_len != bit_len * in_len / (8 * in_width)) throw std::invalid_argument("CompressArray out_len");
    const uint32_t mask = (1u << bit_len) - 1;
    uint64_t acc = 0;
    size_t acc_bits = 0, j = 0;
    for (size_t i = 0; i < out_len; ++i) {
        while (acc_bits < 8) {
            uint32_t v = 0;
            for (size_t b = byte_pad; b < in_width; ++b) v = (v << 8) | in[j + b];
            acc = (acc << bit_len) | (v & mask);
            acc_bits += bit_len;
            j += in_width;
        }
        acc_bits -= 8;
        out[i] = (unsigned char)(acc >> acc_bits);
    }
}

std::vector<uint32_t> GetIndicesFromMinimal(const std::vector<unsigned char>& minimal, size_t cBitLen) {
    const size_t bits = cBitLen + 1;
    const size_t n = 8 * minimal.size() / bits;
    std::vector<uint32_t> ret(n);
    uint64_t acc = 0;
    size_t acc_bits = 0, pos = 0;
    for (size_t i = 0; i < n; ++i) {
        while (acc_bits < bits) {
            acc = (acc << 8) | minimal[pos++];
            acc_bits += 8;
        }
        ret[i] = (uint32_t)(acc >> (acc_bits - bits)) & ((1u << bits) - 1);
        acc_bits -= bits;
    }
    return ret;
}

std::vector<unsigned char> GetMinimalFromIndices(const std::vector<uint32_t>& indices, size_t cBitLen) {
    const size_t bits = cBitLen + 1;
    std::vector<unsigned char> ret(bits * indices.size() / 8);
    uint64_t acc = 0;
    size_t acc_bits = 0, pos = 0;
    for (uint32_t v : indices) {
        acc = (acc << bits) | (v & ((1u << bits) - 1));
        acc_bits += bits;
        while (acc_bits >= 8) {
            acc_bits -= 8;
            ret[pos++] = (unsigned char)(acc >> acc_bits);
        }
    }
    return ret;
}

namespace {
// Split the (N/8)-byte slice of a digest into K+1 digits of CBL bits.
void HashToDigits(const EquihashParams& p, const unsigned char* slice, uint32_t* digits) {
    const unsigned cbl = p.CollisionBitLength();
    uint64_t acc = 0;
    unsigned acc_bits = 0, pos = 0;
    for (unsigned d = 0; d <= p.K; ++d) {
        while (acc_bits < cbl) {
            acc = (acc << 8) | slice[pos++];
            acc_bits += 8;
        }
        digits[d] = (uint32_t)(acc >> (acc_bits - cbl)) & ((1u << cbl) - 1);
        acc_bits -= cbl;
    }
}

bool LexLess(const uint32_t* a, const uint32_t* b, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        if (a[i] != b[i]) return a[i] < b[i];
    }
    return false;
}
} // namespace

bool EhIsValidSolution(const EquihashParams& p, const CBlake2b& base, const std::vector<unsigned char>& soln,
                       std::string* reason) {
    auto fail = [&](const char* r) {
        if (reason) *reason = r;
        return false;
    };
    if (!p.Valid()) return fail("bad-params");
    if (soln.size() != p.SolutionWidth()) return fail("invalid-solution-length");
    const unsigned cbl = p.CollisionBitLength();
    const unsigned D = p.K + 1;
    std::vector<uint32_t> idx = GetIndicesFromMinimal(soln, cbl);
    const size_t L = idx.size(); // 2^K
    std::vector<uint32_t> dig(L * D);
    std::vector<unsigned char> h(p.HashOutput());
    const unsigned iph = p.IndicesPerHashOutput();
    for (size_t i = 0; i < L; ++i) {
        EhGenerateHash(base, idx[i] / iph, h.data());
        HashToDigits(p, h.data() + (idx[i] % iph) * (p.N / 8), &dig[i * D]);
    }
    // Merge level by level; node j at level l owns leaves [j*2^l, (j+1)*2^l) and
    // its digits are stored in place of its first leaf.
    for (unsigned l = 0; l < p.K; ++l) {
        const size_t w = (size_t)1 << l;
        for (size_t j = 0; j < L; j += 2 * w) {
            uint32_t* a = &dig[j * D];
            uint32_t* b = &dig[(j + w) * D];
            if (a[l] != b[l]) return fail("invalid-collision");
            if (LexLess(&idx[j + w], &idx[j], w)) return fail("index-tree-incorrectly-ordered");
            // distinct indices between the two halves
            for (size_t x = 0; x < w; ++x)
                for (size_t y = 0; y < w; ++y)
                    if (idx[j + x] == idx[j + w + y]) return fail("duplicate-indices");
            for (unsigned d = l; d < D; ++d) a[d] ^= b[d];
        }
    }
    if (dig[p.K] != 0) return fail("nonzero-final-xor");
    return true;
}

bool EhCanonicaliseIndices(std::vector<uint32_t>& idx, unsigned K) {
    const size_t L = (size_t)1 << K;
    if (idx.size() != L) return false;
    std::vector<uint32_t> tmp(L);
    for (unsigned l = 0; l < K; ++l) {
        const size_t w = (size_t)1 << l;
        for (size_t j = 0; j < L; j += 2 * w) {
            if (LexLess(&idx[j + w], &idx[j], w)) {
                std::copy(idx.begin() + j, idx.begin() + j + w, tmp.begin());
                std::copy(idx.begin() + j + w, idx.begin() + j + 2 * w, idx.begin() + j);
                std::copy(tmp.begin(), tmp.begin() + w, idx.begin() + j + w);
            }
        }
    }
    std::vector<uint32_t> s(idx);
    std::sort(s.begin(), s.end());
    return std::adjacent_find(s.begin(), s.end()) == s.end();
}

bool EhBasicSolve(const EquihashParams& p, const CBlake2b& base,
                  const std::function<bool(const std::vector<unsigned char>&)>& validBlock,
                  const std::function<bool()>& cancelled, EhSolveStats* stats) {
    if (!p.Valid()) throw std::invalid_argument("bad equihash params");
    const unsigned cbl = p.CollisionBitLength();
    const unsigned D = p.K + 1;
    const uint32_t init = p.InitSize();
    const unsigned iph = p.IndicesPerHashOutput();

    // Round 0 rows: all digits, parent reference = leaf index.
    std::vector<uint32_t> cur((size_t)init * D);
    std::vector<unsigned char> h(p.HashOutput());
    for (uint32_t g = 0; g * iph < init; ++g) {
        EhGenerateHash(base, g, h.data());
        for (unsigned s = 0; s < iph && g * iph + s < init; ++s)
            HashToDigits(p, h.data() + s * (p.N / 8), &cur[(size_t)(g * iph + s) * D]);
    }
    if (cancelled && cancelled()) return false;
    // refs[r][i] = (a<<32)|b : row i of round r merges rows a,b of round r-1.
    std::vector<std::vector<uint64_t>> refs(p.K);
    size_t nrows = init;
    unsigned width = D; // digits per row in `cur`; row digit 0 == global digit (D - width)

    std::vector<std::pair<uint64_t, uint32_t>> order;
    for (unsigned r = 1; r < p.K; ++r) {
        order.resize(nrows);
        for (size_t i = 0; i < nrows; ++i) order[i] = {cur[i * width], (uint32_t)i};
        std::sort(order.begin(), order.end());
        std::vector<uint32_t> next;
        std::vector<uint64_t>& ref = refs[r];
        ref.clear();
        const unsigned nw = width - 1;
        next.reserve(nrows * nw);
        for (size_t i = 0; i < nrows;) {
            size_t j = i + 1;
            while (j < nrows && order[j].first == order[i].first) ++j;
            for (size_t a = i; a < j; ++a) {
                for (size_t b = a + 1; b < j; ++b) {
                    if (r >= 2) {
                        // Depth-1 duplicate pruning: rows sharing a parent row merge to a tree
                        // with repeated leaves (cheap early reject, as on the GPU).
                        const uint64_t pa = refs[r - 1][order[a].second], pb = refs[r - 1][order[b].second];
                        const uint32_t a0 = (uint32_t)(pa >> 32), a1 = (uint32_t)pa, b0 = (uint32_t)(pb >> 32),
                                       b1 = (uint32_t)pb;
                        if (a0 == b0 || a0 == b1 || a1 == b0 || a1 == b1) continue;
                    }
                    const uint32_t* ra = &cur[(size_t)order[a].second * width];
                    const uint32_t* rb = &cur[(size_t)order[b].second * width];
                    bool allzero = true;
                    size_t base_off = next.size();
                    for (unsigned d = 1; d < width; ++d) {
                        uint32_t x = ra[d] ^ rb[d];
                        allzero &= (x == 0);
                        next.push_back(x);
                    }
                    if (allzero) { // identical subtrees -> duplicate indices
                        next.resize(base_off);
                        continue;
                    }
                    ref.push_back(((uint64_t)order[a].second << 32) | order[b].second);
                }
            }
            i = j;
        }
        cur.swap(next);
        nrows = ref.size();
        width = nw;
        if (cancelled && cancelled()) return false;
    }
    // Final round: collide on the last two digits.
    assert(width == 2);
    order.resize(nrows);
    for (size_t i = 0; i < nrows; ++i) order[i] = {((uint64_t)cur[i * 2] << cbl) | cur[i * 2 + 1], (uint32_t)i};
    std::sort(order.begin(), order.end());
    const size_t L = (size_t)1 << p.K;
    for (size_t i = 0; i < nrows;) {
        size_t j = i + 1;
        while (j < nrows && order[j].first == order[i].first) ++j;
        for (size_t a = i; a < j; ++a) {
            for (size_t b = a + 1; b < j; ++b) {
                {
                    const uint64_t pa = refs[p.K - 1][order[a].second], pb = refs[p.K - 1][order[b].second];
                    const uint32_t a0 = (uint32_t)(pa >> 32), a1 = (uint32_t)pa, b0 = (uint32_t)(pb >> 32),
                                   b1 = (uint32_t)pb;
                    if (a0 == b0 || a0 == b1 || a1 == b0 || a1 == b1) {
                        if (stats) stats->duplicates++;
                        continue;
                    }
                }
                if (stats) stats->candidates++;
                // Expand the tree top-down.
                std::vector<uint32_t> nodes = {order[a].second, order[b].second};
                for (int r = (int)p.K - 1; r >= 1; --r) {
                    std::vector<uint32_t> child(nodes.size() * 2);
                    for (size_t x = 0; x < nodes.size(); ++x) {
                        uint64_t rr = refs[r][nodes[x]];
                        child[2 * x] = (uint32_t)(rr >> 32);
                        child[2 * x + 1] = (uint32_t)rr;
                    }
                    nodes.swap(child);
                }
                assert(nodes.size() == L);
                if (!EhCanonicaliseIndices(nodes, p.K)) {
                    if (stats) stats->duplicates++;
                    continue;
                }
                if (stats) stats->solutions++;
                if (validBlock(GetMinimalFromIndices(nodes, cbl))) return true;
            }
        }
        i = j;
        if (cancelled && cancelled()) return false;
    }
    return false;
}

std::vector<std::vector<unsigned char>> EhSolveAll(const EquihashParams& p, const CBlake2b& base,
                                                   EhSolveStats* stats) {
    std::vector<std::vector<unsigned char>> out;
    EhBasicSolve(p, base, [&](const std::vector<unsigned char>& s) { out.push_back(s); return false; }, nullptr,
                 stats);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

} // namespace bcp
