"""Deserialization fuzzing (reference src/test/test_bitcoin_fuzzy.cpp, doc/fuzzing.md): every
bcp-fuzz target is fed seeded, mutated inputs (bit flips, truncation, splices, length-field
corruption) built from real serializations; the harness must exit cleanly on all of them
(caught parse errors only: no crash, abort, sanitizer report or hang)."""
import os
import random
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "bin", "bcp-fuzz")
FUZZ_ASAN = os.path.join(ROOT, "bin", "bcp-fuzz-asan")  # `make asan` (host ASan+UBSan build)
BLOCK = os.path.join(ROOT, "bench", "data", "block413567.raw")

if not os.path.exists(FUZZ):
    subprocess.check_call(["make", "-C", ROOT, "-j8", "bin/bcp-fuzz"])


def targets():
    return subprocess.run([FUZZ, "-list"], capture_output=True, text=True, check=True).stdout.split()


def seeds():
    raw = open(BLOCK, "rb").read()
    header = raw[:80]
    # transactions start after the header and the CompactSize count (0xfd + u16 here)
    off = 80 + (3 if raw[80] == 0xFD else 1)
    new_header = header[:4] + raw[4:68] + struct.pack("<I", 3000) + bytes(28) + header[68:80] + bytes(32) + b"\x00"
    return {
        "block_legacy": [raw],
        "block": [new_header + raw[80:]],
        "block_header": [new_header, header],
        "transaction": [raw[off:off + 400], raw[off:]],
        "equihash_solution": [bytes(36), bytes(1344)],
        "script_eval": [b"\x00\x00\x00\x00" + bytes([0x51, 0x52, 0x93, 0x53, 0x87]), b"\xff\xff\xff\xff" + b"\x76\xa9"],
        "bloom_filter": [b"\x04\xff\xff\xff\xff\x05\x00\x00\x00\x01\x00\x00\x00\x01"],
        "address": [struct.pack("<IQ", 1, 1) + bytes(10) + b"\xff\xff\x7f\x00\x00\x01" + b"\x20\x8d"],
        "inv": [struct.pack("<I", 2) + bytes(32)],
    }


def mutate(rng, data):
    b = bytearray(data)
    for _ in range(rng.randint(1, 6)):
        op = rng.randrange(5)
        if op == 0 and b:  # bit flip
            i = rng.randrange(len(b))
            b[i] ^= 1 << rng.randrange(8)
        elif op == 1 and b:  # truncate
            del b[rng.randrange(len(b)):]
        elif op == 2:  # insert random bytes
            i = rng.randrange(len(b) + 1)
            b[i:i] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 16)))
        elif op == 3 and len(b) > 4:  # huge length prefix (CompactSize 0xfe / 0xff)
            i = rng.randrange(len(b))
            b[i:i + 1] = rng.choice([b"\xfd\xff\xff", b"\xfe\xff\xff\xff\x7f", b"\xff" + bytes([0xff] * 8)])
        elif op == 4 and len(b) > 8:  # duplicate a slice
            i = rng.randrange(len(b) - 4)
            b[i:i] = b[i:i + rng.randint(1, 64)]
    return bytes(b)


def corpus(target, tmp_path, count=150):
    rng = random.Random(f"bcp-fuzz-{target}")
    base = seeds().get(target, []) + [b"", bytes(64), bytes(rng.randrange(256) for _ in range(300))]
    files = []
    for i in range(count):
        data = mutate(rng, rng.choice(base)) if i else base[0]
        p = tmp_path / f"in{i}"
        p.write_bytes(data)
        files.append(str(p))
    return files


@pytest.mark.parametrize("target", targets())
def test_fuzz_target_survives_mutations(target, tmp_path):
    r = subprocess.run([FUZZ, f"-target={target}"] + corpus(target, tmp_path), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(FUZZ_ASAN), reason="host sanitizer build not present (make asan)")
@pytest.mark.parametrize("target", targets())
def test_fuzz_target_clean_under_asan_ubsan(target, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([FUZZ_ASAN, f"-target={target}"] + corpus(target, tmp_path, 60), capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-3000:]


def test_selector_mode_from_stdin():
    # AFL-style: first 4 bytes pick the target, input on stdin
    n = len(targets())
    for sel in range(n):
        r = subprocess.run([FUZZ], input=struct.pack("<I", sel) + bytes(range(200)), capture_output=True, timeout=60)
        assert r.returncode == 0
