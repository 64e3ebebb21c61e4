"""Host emulation of the device secp256k1 field arithmetic (csrc/kernels/secp256k1.hip).

The kernel keeps field elements lazily reduced (any value below 2^256, folded with
2^256 = 2^32 + 977 mod p) and multiplies by product scanning on v_mad_u64_u32 with carry-out.
This test extracts the field functions from the kernel source verbatim, replaces the one inline-asm
step (fe_mac: {acc} += a*b, carry into c2) with its 128-bit host equivalent, compiles them with
clang on the CPU, and checks products, squares, sums, differences and small multiples against
Python integers mod p, including the lazily reduced inputs in [p, 2^256) the kernel produces.
The GPU path is covered end to end by tests/test_ecdsa_batch.py and the 10k differential test
(tests/test_gpu_verify_service.py); this one pins the arithmetic without a GPU.
"""
import os
import random
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**256 - 2**32 - 977
CLANG = "/opt/rocm/llvm/bin/clang++"


def _harness(tmp):
    src = open(os.path.join(ROOT, "csrc/kernels/secp256k1.hip")).read()
    body = src[src.index("__device__ __constant__ uint32_t P_LIMBS[8]"):
               src.index("__device__ __forceinline__ void fe_sqr_n(fe& r, const fe& a, int n) {")]
    body = (body.replace("__device__ __constant__", "static const")
            .replace("__device__ __forceinline__", "static inline")
            .replace("__device__ __noinline__", "static"))
    body, n = re.subn(r"static inline void fe_mac\(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b\) \{.*?\n\}\n",
                      "static inline void fe_mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {\n"
                      "    unsigned __int128 s = (unsigned __int128)a * b + acc;\n"
                      "    acc = (uint64_t)s;\n    c2 += (uint32_t)(s >> 64);\n}\n", body, flags=re.S)
    assert n == 1, "fe_mac not found in the kernel source"
    body = body.replace("__builtin_amdgcn_alignbit(t[i], t[i - 1], 31)", "((t[i] << 1) | (t[i - 1] >> 31))")
    prog = ("#include <cstdint>\n#include <cstdio>\n#include <cstdlib>\nstruct fe { uint32_t v[8]; };\n" + body + r"""
static bool rd(fe& a) { for (int i = 0; i < 8; i++) { unsigned x; if (scanf("%x", &x) != 1) return false; a.v[i] = x; } return true; }
int main() {
    int op;
    while (scanf("%d", &op) == 1) {
        fe a, b, r;
        if (!rd(a) || !rd(b)) return 1;
        if (op == 0) fe_mul_impl(r, a, b);
        else if (op == 1) fe_sqr_impl(r, a);
        else if (op == 2) fe_add(r, a, b);
        else if (op == 3) fe_sub(r, a, b);
        else fe_mul_small(r, a, b.v[0]);
        for (int i = 0; i < 8; i++) printf("%08x ", r.v[i]);
        printf("\n");
    }
    return 0;
}
""")
    c = os.path.join(tmp, "fe_host.cpp")
    exe = os.path.join(tmp, "fe_host")
    open(c, "w").write(prog)
    subprocess.run([CLANG, "-O1", "-std=c++17", c, "-o", exe], check=True, capture_output=True)
    return exe


@pytest.mark.skipif(not shutil.which(CLANG) and not os.path.exists(CLANG), reason="clang not available")
def test_device_field_arithmetic_matches_python(tmp_path):
    exe = _harness(str(tmp_path))
    rng = random.Random(7)
    special = [0, 1, 2, P - 1, P, P + 1, P + 977, 2**256 - 1, 2**256 - 2, 2**255, 2**224, 2**256 - 2**32,
               2**256 - 2**32 - 977 - 1] + [P + rng.randrange(2**32 + 977) for _ in range(16)]
    special = [v for v in special if v < 2**256]

    def pick():
        return rng.choice(special) if rng.random() < 0.35 else rng.getrandbits(256)

    cases = []
    for _ in range(12000):
        op = rng.randrange(5)
        a, b = pick(), pick()
        if op == 4:
            b = rng.choice([2, 3, 4, 8])
        cases.append((op, a, b))

    def limbs(x):
        return " ".join("%x" % ((x >> (32 * i)) & 0xFFFFFFFF) for i in range(8))

    out = subprocess.run([exe], input="".join(f"{op} {limbs(a)} {limbs(b)}\n" for op, a, b in cases),
                         capture_output=True, text=True, check=True).stdout.split("\n")
    for (op, a, b), line in zip(cases, out):
        r = sum(int(x, 16) << (32 * i) for i, x in enumerate(line.split()))
        want = [a * b, a * a, a + b, a - b, a * b][op] % P
        assert r < 2**256 and r % P == want, (op, hex(a), hex(b), hex(r))
