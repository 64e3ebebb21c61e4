// Lax DER signature parsing for the ECDSA prep kernel, host-compilable so the host unit test
// (csrc/test/derlax_tests.cpp) can compare it with the CPU parser (secp::sig_parse_der_lax).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define BCP_DERLAX_HD __host__ __device__
#else
#define BCP_DERLAX_HD
#endif

namespace bcpk {

// Lax DER parse on the device (the reference's ecdsa_signature_parse_der_lax, src/pubkey.cpp,
// as secp::sig_parse_der_lax on the host): false if the encoding cannot be walked; otherwise
// r and s as 32-byte big-endian values, both zero when either does not fit in 32 bytes.
BCP_DERLAX_HD inline bool der_lax_parse(const unsigned char* in, uint32_t len, unsigned char out[64]) {
    for (int i = 0; i < 64; i++) out[i] = 0;
    uint32_t pos = 0;
    if (pos == len || in[pos] != 0x30) return false;
    pos++;
    if (pos == len) return false;
    uint32_t lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (pos + lenbyte > len) return false;
        pos += lenbyte;
    }
    uint32_t ipos[2], ilen[2];
    for (int k = 0; k < 2; k++) {
        if (pos == len || in[pos] != 0x02) return false;
        pos++;
        if (pos == len) return false;
        lenbyte = in[pos++];
        uint64_t l;
        if (lenbyte & 0x80) {
            lenbyte -= 0x80;
            if (pos + lenbyte > len) return false;
            while (lenbyte > 0 && in[pos] == 0) {
                pos++;
                lenbyte--;
            }
            if (lenbyte >= 8) return false;
            l = 0;
            while (lenbyte > 0) {
                l = (l << 8) + in[pos];
                pos++;
                lenbyte--;
            }
        } else {
            l = lenbyte;
        }
        if (l > (uint64_t)(len - pos)) return false;
        ipos[k] = pos;
        ilen[k] = (uint32_t)l;
        pos += (uint32_t)l;
    }
    bool overflow = false;
    for (int k = 0; k < 2; k++) {
        while (ilen[k] > 0 && in[ipos[k]] == 0) {
            ilen[k]--;
            ipos[k]++;
        }
        if (ilen[k] > 32) overflow = true;
    }
    if (!overflow)
        for (int k = 0; k < 2; k++)
            for (uint32_t b = 0; b < ilen[k]; b++) out[32 * k + 32 - ilen[k] + b] = in[ipos[k] + b];
    return true;
}


} // namespace bcpk
