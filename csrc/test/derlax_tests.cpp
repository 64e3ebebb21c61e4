// derlax_tests: the ECDSA prep kernel's lax DER parser (csrc/kernels/der_lax.h), run on the host
// against the CPU parser (bcp::secp::sig_parse_der_lax, the reference's ecdsa_signature_parse_der_lax
// in src/pubkey.cpp) over valid encodings and randomly mutated ones.
#include "test/unittest.h"

#include "kernels/der_lax.h"
#include "secp256k1/secp256k1.h"

#include <cstring>
#include <random>
#include <vector>

namespace {

const unsigned char N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                                0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};

bool GeN(const unsigned char* v) { return memcmp(v, N_BE, 32) >= 0; }

std::vector<unsigned char> Int(std::mt19937_64& rng, bool pad) {
    std::vector<unsigned char> v(1 + rng() % 33);
    for (auto& b : v) b = (unsigned char)rng();
    if (pad && !v.empty()) v.insert(v.begin(), 0);
    return v;
}

std::vector<unsigned char> Der(const std::vector<unsigned char>& r, const std::vector<unsigned char>& s) {
    std::vector<unsigned char> o{0x30, (unsigned char)(4 + r.size() + s.size()), 0x02, (unsigned char)r.size()};
    o.insert(o.end(), r.begin(), r.end());
    o.push_back(0x02);
    o.push_back((unsigned char)s.size());
    o.insert(o.end(), s.begin(), s.end());
    return o;
}

} // namespace

TEST_CASE(derlax_tests, device_parser_matches_cpu) {
    std::mt19937_64 rng(77);
    int mismatch = 0, parsed = 0, total = 0;
    for (int t = 0; t < 200000; t++) {
        std::vector<unsigned char> d = Der(Int(rng, rng() & 1), Int(rng, rng() & 1));
        // mutations: flip / insert / delete bytes, long-form lengths, truncation, trailing data
        const int muts = (int)(rng() % 4);
        for (int m = 0; m < muts && !d.empty(); m++) {
            const size_t at = rng() % d.size();
            switch (rng() % 6) {
            case 0: d[at] ^= (unsigned char)(1u << (rng() % 8)); break;
            case 1: d.insert(d.begin() + at, (unsigned char)rng()); break;
            case 2: d.erase(d.begin() + at); break;
            case 3: d[at] = (unsigned char)(0x80 | (rng() % 9)); break; // a long-form length byte
            case 4: d.resize(at); break;
            case 5: d.push_back((unsigned char)rng()); break;
            }
        }
        if (d.size() > 72) d.resize(72); // a deferred check carries at most 72 bytes
        total++;
        bcp::secp::Signature cs;
        const bool cok = bcp::secp::sig_parse_der_lax(cs, d.data(), d.size());
        unsigned char dv[64];
        const bool dok = bcpk::der_lax_parse(d.data(), (uint32_t)d.size(), dv);
        if (cok != dok) {
            mismatch++;
            continue;
        }
        if (!cok) continue;
        parsed++;
        // the CPU parser zeroes the signature when r or s is >= n; the prep kernel's range check
        // rejects those values the same way
        unsigned char want[64];
        bcp::secp::sig_serialize_compact(want, cs);
        unsigned char got[64];
        memcpy(got, dv, 64);
        if (GeN(got) || GeN(got + 32)) memset(got, 0, 64);
        if (memcmp(want, got, 64) != 0) mismatch++;
    }
    CHECK_EQ(mismatch, 0);
    CHECK(parsed > total / 10); // the mutations leave plenty of parseable encodings
}
