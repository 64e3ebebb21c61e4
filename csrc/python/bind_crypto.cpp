// Python bindings: hash primitives, big integers, Equihash CPU reference.
#include "consensus/equihash.h"
#include "crypto/hashes.h"
#include "primitives/uint256.h"
#include "python/bind.h"
#include "util/strencodings.h"

namespace bcp {
namespace py {

void bind_crypto(pyb::module_& m) {
    m.def("sha256", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[32];
        Sha256(v.data(), v.size(), out);
        return to_bytes(out, 32);
    });
    m.def("sha256d", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[32];
        Sha256d(v.data(), v.size(), out);
        return to_bytes(out, 32);
    });
    m.def("sha512", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[64];
        CSHA512().Write(v.data(), v.size()).Finalize(out);
        return to_bytes(out, 64);
    });
    m.def("sha1", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[20];
        CSHA1().Write(v.data(), v.size()).Finalize(out);
        return to_bytes(out, 20);
    });
    m.def("ripemd160", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[20];
        CRIPEMD160().Write(v.data(), v.size()).Finalize(out);
        return to_bytes(out, 20);
    });
    m.def("hash160", [](const pyb::bytes& b) {
        auto v = to_vec(b);
        unsigned char out[20];
        Hash160(v.data(), v.size(), out);
        return to_bytes(out, 20);
    });
    m.def("hmac_sha256", [](const pyb::bytes& key, const pyb::bytes& b) {
        auto k = to_vec(key), v = to_vec(b);
        unsigned char out[32];
        CHMAC_SHA256(k.data(), k.size()).Write(v.data(), v.size()).Finalize(out);
        return to_bytes(out, 32);
    });
    m.def("hmac_sha512", [](const pyb::bytes& key, const pyb::bytes& b) {
        auto k = to_vec(key), v = to_vec(b);
        unsigned char out[64];
        CHMAC_SHA512(k.data(), k.size()).Write(v.data(), v.size()).Finalize(out);
        return to_bytes(out, 64);
    });
    m.def(
        "blake2b",
        [](const pyb::bytes& b, size_t outlen, const pyb::bytes& key, const pyb::bytes& salt,
           const pyb::bytes& person) {
            auto v = to_vec(b), k = to_vec(key), s = to_vec(salt), p = to_vec(person);
            s.resize(16, 0);
            p.resize(16, 0);
            CBlake2b h(outlen, k.empty() ? nullptr : k.data(), k.size(), s.data(), p.data());
            h.Write(v.data(), v.size());
            std::vector<unsigned char> out(outlen);
            h.Finalize(out.data());
            return to_bytes(out);
        },
        pyb::arg("data"), pyb::arg("digest_size") = 64, pyb::arg("key") = pyb::bytes(""),
        pyb::arg("salt") = pyb::bytes(""), pyb::arg("person") = pyb::bytes(""));
    m.def("siphash", [](uint64_t k0, uint64_t k1, const pyb::bytes& b) {
        auto v = to_vec(b);
        return CSipHasher(k0, k1).Write(v.data(), v.size()).Finalize();
    });
    m.def("siphash_uint256", [](uint64_t k0, uint64_t k1, const pyb::bytes& b) {
        auto v = to_vec(b);
        if (v.size() != 32) throw std::invalid_argument("need 32 bytes");
        return SipHashUint256(k0, k1, v.data());
    });
    m.def("siphash_uint256_extra", [](uint64_t k0, uint64_t k1, const pyb::bytes& b, uint32_t extra) {
        auto v = to_vec(b);
        if (v.size() != 32) throw std::invalid_argument("need 32 bytes");
        return SipHashUint256Extra(k0, k1, v.data(), extra);
    });
    m.def("chacha20", [](const pyb::bytes& key, uint64_t iv, uint64_t seek, size_t n) {
        auto k = to_vec(key);
        ChaCha20 c(k.data(), k.size());
        c.SetIV(iv);
        c.Seek(seek);
        std::vector<unsigned char> out(n);
        c.Output(out.data(), n);
        return to_bytes(out);
    });
    m.def("aes256cbc_encrypt", [](const pyb::bytes& key, const pyb::bytes& iv, const pyb::bytes& data, bool pad) {
        auto k = to_vec(key), i = to_vec(iv), d = to_vec(data);
        if (k.size() != 32 || i.size() != 16) throw std::invalid_argument("key/iv size");
        std::vector<unsigned char> out(d.size() + 16);
        int n = AES256CBCEncrypt(k.data(), i.data(), pad).Encrypt(d.data(), (int)d.size(), out.data());
        out.resize(n);
        return to_bytes(out);
    });
    m.def("aes256cbc_decrypt", [](const pyb::bytes& key, const pyb::bytes& iv, const pyb::bytes& data, bool pad) {
        auto k = to_vec(key), i = to_vec(iv), d = to_vec(data);
        if (k.size() != 32 || i.size() != 16) throw std::invalid_argument("key/iv size");
        std::vector<unsigned char> out(d.size());
        int n = AES256CBCDecrypt(k.data(), i.data(), pad).Decrypt(d.data(), (int)d.size(), out.data());
        out.resize(n);
        return to_bytes(out);
    });
    // Compact difficulty encoding on hex strings.
    m.def("compact_to_target_hex", [](uint32_t c) {
        bool neg = false, ovf = false;
        arith_uint256 t;
        t.SetCompact(c, &neg, &ovf);
        return pyb::make_tuple(t.GetHex(), neg, ovf);
    });
    m.def("target_hex_to_compact", [](const std::string& hex, bool negative) {
        arith_uint256 t(hex);
        return t.GetCompact(negative);
    }, pyb::arg("hex"), pyb::arg("negative") = false);
    m.def("uint256_from_hex", [](const std::string& hex) {
        uint256 u = uint256S(hex);
        return to_bytes(u.begin(), 32);
    });
}

void bind_equihash(pyb::module_& m) {
    pyb::class_<CBlake2b>(m, "EquihashState")
        .def(pyb::init([](unsigned n, unsigned k) { return EhInitialiseState(EquihashParams(n, k)); }))
        .def("update", [](CBlake2b& s, const pyb::bytes& b) {
            auto v = to_vec(b);
            s.Write(v.data(), v.size());
        })
        .def("copy", [](const CBlake2b& s) { return CBlake2b(s); })
        .def("hash", [](const CBlake2b& s, uint32_t g) {
            std::vector<unsigned char> out(s.OutLen());
            EhGenerateHash(s, g, out.data());
            return to_bytes(out);
        })
        .def("state_bytes", [](const CBlake2b& s) {
            const Blake2bState& st = s.GetState();
            return to_bytes((const unsigned char*)&st, sizeof(st));
        });
    m.def("eh_solution_width", [](unsigned n, unsigned k) { return EquihashParams(n, k).SolutionWidth(); });
    m.def("eh_is_valid_solution", [](unsigned n, unsigned k, const CBlake2b& base, const pyb::bytes& soln) {
        std::string reason;
        bool ok = EhIsValidSolution(EquihashParams(n, k), base, to_vec(soln), &reason);
        return pyb::make_tuple(ok, reason);
    });
    m.def("eh_solve_cpu", [](unsigned n, unsigned k, const CBlake2b& base) {
        EhSolveStats st;
        std::vector<std::vector<unsigned char>> sols;
        {
            pyb::gil_scoped_release rel;
            sols = EhSolveAll(EquihashParams(n, k), base, &st);
        }
        pyb::list out;
        for (auto& s : sols) out.append(to_bytes(s));
        pyb::dict stats;
        stats["candidates"] = st.candidates;
        stats["duplicates"] = st.duplicates;
        stats["solutions"] = st.solutions;
        return pyb::make_tuple(out, stats);
    });
    m.def("eh_indices_from_minimal", [](const pyb::bytes& b, size_t cbl) {
        return GetIndicesFromMinimal(to_vec(b), cbl);
    });
    m.def("eh_minimal_from_indices", [](const std::vector<uint32_t>& idx, size_t cbl) {
        return to_bytes(GetMinimalFromIndices(idx, cbl));
    });
    m.def("eh_expand_array", [](const pyb::bytes& in, size_t bit_len, size_t byte_pad) {
        auto v = to_vec(in);
        size_t groups = 8 * v.size() / bit_len;
        size_t w = (bit_len + 7) / 8 + byte_pad;
        std::vector<unsigned char> out(groups * w);
        ExpandArray(v.data(), v.size(), out.data(), out.size(), bit_len, byte_pad);
        return to_bytes(out);
    });
    m.def("eh_compress_array", [](const pyb::bytes& in, size_t bit_len, size_t byte_pad) {
        auto v = to_vec(in);
        size_t w = (bit_len + 7) / 8 + byte_pad;
        std::vector<unsigned char> out(bit_len * v.size() / (8 * w));
        CompressArray(v.data(), v.size(), out.data(), out.size(), bit_len, byte_pad);
        return to_bytes(out);
    });
}

} // namespace py
} // namespace bcp
