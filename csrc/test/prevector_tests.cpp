// prevector (util/prevector.h), the storage of CScript.
// Parity: reference src/test/prevector_tests.cpp (randomised operations on a prevector and a
// std::vector side by side, every state compared). Here the element type is the one CScript
// uses, the inline size is 28 as for scripts plus a tiny one (4) so that the inline -> heap and
// heap -> inline transitions happen constantly, and the serialised form is compared too.
#include "test/unittest.h"

#include "primitives/serialize.h"
#include "script/script.h"
#include "util/memusage.h"
#include "util/prevector.h"

#include <random>
#include <vector>

using namespace bcp;

namespace {

template <unsigned N> struct Pair {
    prevector<N, unsigned char> p;
    std::vector<unsigned char> v;
    bool Same() const {
        if (p.size() != v.size() || p.empty() != v.empty()) return false;
        if (!std::equal(p.begin(), p.end(), v.begin(), v.end())) return false;
        if (p.capacity() < p.size()) return false;
        if (!v.empty() && (p.front() != v.front() || p.back() != v.back())) return false;
        for (size_t i = 0; i < v.size(); i++)
            if (p[(uint32_t)i] != v[i]) return false;
        // reverse iteration and the byte serialisation agree with the std::vector's
        if (!std::equal(p.rbegin(), p.rend(), v.rbegin(), v.rend())) return false;
        return SerializeToBytes(p) == SerializeToBytes(v);
    }
};

template <unsigned N> void RandomOps(uint64_t seed) {
    std::mt19937_64 rng(seed);
    Pair<N> x;
    for (int step = 0; step < 4000; step++) {
        const unsigned op = rng() % 17;
        const unsigned char val = (unsigned char)rng();
        const uint32_t sz = x.p.size();
        switch (op) {
        case 0: { // resize (grow zero-filled or shrink)
            const uint32_t n = rng() % (3 * N + 8);
            x.p.resize(n);
            x.v.resize(n);
            break;
        }
        case 1: { // insert one
            const uint32_t at = sz ? rng() % (sz + 1) : 0;
            x.p.insert(x.p.begin() + at, val);
            x.v.insert(x.v.begin() + at, val);
            break;
        }
        case 2: { // insert n copies
            const uint32_t at = sz ? rng() % (sz + 1) : 0, n = rng() % (N + 3);
            x.p.insert(x.p.begin() + at, n, val);
            x.v.insert(x.v.begin() + at, n, val);
            break;
        }
        case 3: { // insert a range from outside
            const uint32_t at = sz ? rng() % (sz + 1) : 0;
            std::vector<unsigned char> src(rng() % (2 * N + 5));
            for (auto& c : src) c = (unsigned char)rng();
            x.p.insert(x.p.begin() + at, src.begin(), src.end());
            x.v.insert(x.v.begin() + at, src.begin(), src.end());
            break;
        }
        case 4: { // insert a range of itself (the source moves while the gap opens)
            if (!sz) break;
            const uint32_t a = rng() % sz, b = a + rng() % (sz - a + 1), at = rng() % (sz + 1);
            const std::vector<unsigned char> copy(x.v.begin() + a, x.v.begin() + b);
            x.p.insert(x.p.begin() + at, x.p.data() + a, x.p.data() + b);
            x.v.insert(x.v.begin() + at, copy.begin(), copy.end());
            break;
        }
        case 5: { // erase one
            if (!sz) break;
            const uint32_t at = rng() % sz;
            x.p.erase(x.p.begin() + at);
            x.v.erase(x.v.begin() + at);
            break;
        }
        case 6: { // erase a range
            if (!sz) break;
            const uint32_t a = rng() % sz, b = a + rng() % (sz - a + 1);
            x.p.erase(x.p.begin() + a, x.p.begin() + b);
            x.v.erase(x.v.begin() + a, x.v.begin() + b);
            break;
        }
        case 7:
            x.p.push_back(val);
            x.v.push_back(val);
            break;
        case 8: // push back an element of itself
            if (sz) {
                const uint32_t at = rng() % sz;
                x.p.push_back(x.p[at]);
                x.v.push_back(x.v[at]);
            }
            break;
        case 9:
            if (sz) {
                x.p.pop_back();
                x.v.pop_back();
            }
            break;
        case 10:
            if (sz) {
                const uint32_t at = rng() % sz;
                x.p[at] = val;
                x.v[at] = val;
            }
            break;
        case 11:
            x.p.reserve(rng() % (4 * N + 8)); // never shrinks, never changes the contents
            break;
        case 12:
            x.p.shrink_to_fit();
            break;
        case 13: { // assign n copies
            const uint32_t n = rng() % (2 * N + 4);
            x.p.assign(n, val);
            x.v.assign(n, val);
            break;
        }
        case 14: { // copy out and back
            prevector<N, unsigned char> c(x.p);
            CHECK(c == x.p);
            x.p = c;
            break;
        }
        case 15: { // move out and back
            prevector<N, unsigned char> m(std::move(x.p));
            CHECK(x.p.empty());
            x.p = std::move(m);
            break;
        }
        case 16: { // swap with another and back
            prevector<N, unsigned char> o(rng() % (2 * N + 2), val);
            const prevector<N, unsigned char> o0 = o;
            x.p.swap(o);
            CHECK(x.p == o0);
            x.p.swap(o);
            CHECK(o == o0);
            break;
        }
        }
        if (!x.Same()) {
            CHECK(false);
            std::printf("  prevector<%u> diverged at step %d (op %u), sizes %u vs %zu\n", N, step, op, x.p.size(),
                        x.v.size());
            return;
        }
        // unserialising the serialised bytes gives the same vector back
        if (step % 97 == 0) {
            prevector<N, unsigned char> back;
            DataStream ds(SerializeToBytes(x.p), SER_NETWORK, PROTOCOL_VERSION);
            ds >> back;
            CHECK(back == x.p);
        }
    }
}

} // namespace

TEST_CASE(prevector_tests, random_ops_match_std_vector) {
    for (uint64_t seed = 1; seed <= 8; seed++) {
        RandomOps<28>(seed);
        RandomOps<4>(seed * 1000 + 7);
    }
}

TEST_CASE(prevector_tests, scripts_inline_up_to_28_bytes) {
    // a P2PKH output script (25 bytes) and a P2SH one (23) stay inside the object: no heap
    // block, so a Coin holding one has no dynamic memory; a 33-byte-key P2PK script (35) does not
    const CScript p2pkh = CScript() << OP_DUP << OP_HASH160 << std::vector<unsigned char>(20, 1) << OP_EQUALVERIFY
                                    << OP_CHECKSIG;
    const CScript p2sh = CScript() << OP_HASH160 << std::vector<unsigned char>(20, 2) << OP_EQUAL;
    const CScript p2pk = CScript() << std::vector<unsigned char>(33, 3) << OP_CHECKSIG;
    CHECK_EQ(p2pkh.size(), (uint32_t)25);
    CHECK_EQ(p2pkh.allocated_memory(), (size_t)0);
    CHECK_EQ(p2sh.allocated_memory(), (size_t)0);
    CHECK(p2pk.allocated_memory() >= 35);
    CHECK_EQ(memusage::DynamicUsage(static_cast<const CScriptBase&>(p2pkh)), (size_t)0);
    CHECK_EQ(sizeof(CScript), (size_t)32);
    // the CScript serialisation is the byte-vector one (compact size + bytes)
    const std::vector<unsigned char> raw(p2pk.begin(), p2pk.end());
    CHECK(SerializeToBytes(p2pk) == SerializeToBytes(raw));
    CScript back;
    DataStream ds(SerializeToBytes(p2pk), SER_NETWORK, PROTOCOL_VERSION);
    ds >> back;
    CHECK(back == p2pk);
}
