#!/usr/bin/env python3
"""Write the blocks of a hash list, in that order, from a node's blk?????.dat files into one
linear file (bootstrap.dat) or a series of them (reference contrib/linearize/linearize-data.py).

    linearize-data.py CONFIG-FILE

CONFIG-FILE keys: input (the node's blocks/ directory), hashlist (from linearize-hashes.py),
output_file (bootstrap.dat) or output (directory for split files), netmagic (hex of the 4-byte
on-disk message start; regtest default), max_out_sz (split size, bytes), file_timestamp.

Each record on disk and in the output is: netmagic (4) || length (LE u32) || serialized block.
Records are matched to the hash list by their header hash alone (no transaction parsing).
"""
import hashlib
import os
import struct
import sys


def read_config(path):
    s = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#") and "=" in line:
                k, v = line.split("=", 1)
                s[k.strip()] = v.strip()
    return s


def read_compact_size(b, off):
    n = b[off]
    if n < 0xFD:
        return n, off + 1
    if n == 0xFD:
        return struct.unpack_from("<H", b, off + 1)[0], off + 3
    if n == 0xFE:
        return struct.unpack_from("<I", b, off + 1)[0], off + 5
    return struct.unpack_from("<Q", b, off + 1)[0], off + 9


def sha256d_hex(b):
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()[::-1].hex()


def header_hash(block):
    """Both candidate hashes of a stored block. Blocks are stored in the 140-byte header format
    (version|prev|merkle|nHeight|reserved[7]|time|bits|nonce256|solution); the block hash is
    SHA256d of that header + solution after the fork, and SHA256d of the legacy 80-byte header
    (version|prev|merkle|time|bits|low 32 nonce bits) before it. The hash list decides which."""
    sol_len, off = read_compact_size(block, 140)
    h_new = sha256d_hex(block[:off + sol_len])
    legacy = block[:68] + block[100:104] + block[104:108] + block[108:112]
    return sha256d_hex(legacy), h_new, struct.unpack_from("<I", block, 68)[0]


def scan_blocks(indir, magic):
    """Yield (hashes, raw block) for every framed record in blk?????.dat order."""
    n = 0
    while True:
        path = os.path.join(indir, "blk%05d.dat" % n)
        if not os.path.exists(path):
            return
        data = open(path, "rb").read()
        off = 0
        while off + 8 <= len(data):
            if data[off:off + 4] != magic:
                nxt = data.find(magic, off + 1)
                if nxt < 0:
                    break
                off = nxt
                continue
            (size,) = struct.unpack_from("<I", data, off + 4)
            block = data[off + 8:off + 8 + size]
            if len(block) < size:
                break
            h_old, h_new, _ = header_hash(block)
            yield (h_old, h_new), block
            off += 8 + size
        n += 1


def linearize(settings):
    magic = bytes.fromhex(settings.get("netmagic", "dab5bffa"))  # regtest on-disk magic
    wanted = [h.strip() for h in open(settings["hashlist"]) if h.strip()]
    pos = {h: i for i, h in enumerate(wanted)}
    found = {}
    for (h_old, h_new), block in scan_blocks(settings["input"], magic):
        for h in (h_new, h_old):
            if h in pos and h not in found:
                found[h] = block
                break
    missing = [h for h in wanted if h not in found]
    if missing:
        raise SystemExit(f"linearize-data: {len(missing)} block(s) not found, first {missing[0]}")
    max_out = int(settings.get("max_out_sz", 1000 * 1000 * 1000))
    out_dir = settings.get("output")
    out_file = settings.get("output_file", "bootstrap.dat")
    idx, written, f = 0, 0, None
    for h in wanted:
        block = found[h]
        rec = magic + struct.pack("<I", len(block)) + block
        if f is None or (out_dir and written + len(rec) > max_out):
            if f:
                f.close()
                idx += 1
            f = open(os.path.join(out_dir, "blk%05d.dat" % idx) if out_dir else out_file, "wb")
            written = 0
        f.write(rec)
        written += len(rec)
    if f:
        f.close()
    return len(wanted)


if __name__ == "__main__":
    if len(sys.argv) != 2:
        print(__doc__, file=sys.stderr)
        sys.exit(1)
    n = linearize(read_config(sys.argv[1]))
    print(f"Done ({n} blocks written)")
