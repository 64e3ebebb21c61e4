"""A reference Berkeley DB wallet.dat found at the wallet path is converted when bcpd starts.

The reference keeps its wallet in a BDB 4.8 btree file (src/wallet/db.h:26); csrc/wallet/
bdbimport.cpp reads the pages without libdb and writes every record into this node's wallet
store, converting the reference's DER-encoded unencrypted keys (src/key.cpp
ec_privkey_export_der) into bare secrets. No libdb is available here, so the file below is
written from the db_page.h layout (master database listing the sub-database "main", an internal
page over the leaves, overflow chains for big items): parity with files written by BDB itself
is unpinned. The node must start, report the import, own the key and dump its private key.
"""
import hashlib
import os
import struct

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.messages import hash160
from bitcoincashplus_amd.utils import secp256k1_ref as ref

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58check(payload: bytes) -> str:
    data = payload + hashlib.sha256(hashlib.sha256(payload).digest()).digest()[:4]
    n = int.from_bytes(data, "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    return "1" * (len(data) - len(data.lstrip(b"\0"))) + s


def ser_bytes(b: bytes) -> bytes:
    assert len(b) < 253
    return bytes([len(b)]) + b


class BdbWriter:
    """Berkeley DB 4.x btree pages (db_page.h): 26-byte page headers, item offsets after them,
    B_KEYDATA items inline, B_OVERFLOW items for big values."""

    def __init__(self, pagesize=4096):
        self.P = pagesize
        self.pages = []

    def new_page(self, ptype):
        pg = bytearray(self.P)
        n = len(self.pages)
        struct.pack_into("<I", pg, 8, n)
        pg[25] = ptype
        self.pages.append(pg)
        return n

    def item(self, v: bytes) -> bytes:
        if 3 + len(v) <= self.P // 4:
            return struct.pack("<HB", len(v), 1) + v
        first, prev, cap = None, None, self.P - 26
        for off in range(0, len(v), cap):
            pg = self.new_page(7)
            chunk = v[off:off + cap]
            struct.pack_into("<H", self.pages[pg], 22, len(chunk))
            self.pages[pg][26:26 + len(chunk)] = chunk
            if first is None:
                first = pg
            else:
                struct.pack_into("<I", self.pages[prev], 16, pg)
            prev = pg
        return struct.pack("<HBBII", 0, 3, 0, first, len(v))

    def place(self, pg, items):
        top, page = self.P, self.pages[pg]
        for i, it in enumerate(items):
            top -= len(it)
            page[top:top + len(it)] = it
            struct.pack_into("<H", page, 26 + 2 * i, top)
        struct.pack_into("<H", page, 20, len(items))

    def meta(self, pg, root, subdbs):
        m = self.pages[pg]
        struct.pack_into("<IIIB", m, 12, 0x053162, 9, self.P, 0)
        m[25] = 9
        struct.pack_into("<I", m, 48, 0x20 if subdbs else 0)
        struct.pack_into("<I", m, 88, root)

    def file(self, recs):
        self.new_page(9)
        mleaf, smeta = self.new_page(5), self.new_page(9)
        leaves, cur, used = [], [], 26
        for k, v in recs:
            a, b = self.item(k), self.item(v)
            if cur and used + 4 + len(a) + len(b) > self.P:
                leaves.append(cur)
                cur, used = [], 26
            cur += [a, b]
            used += 4 + len(a) + len(b)
        leaves.append(cur)
        leaf_pages = []
        for items in leaves:
            pg = self.new_page(5)
            self.place(pg, items)
            leaf_pages.append(pg)
        root = self.new_page(3)
        self.pages[root][24] = 2
        self.place(root, [struct.pack("<HBBII", 0, 1, 0, c, 0) for c in leaf_pages])
        self.meta(smeta, root, False)
        self.place(mleaf, [self.item(b"main"), self.item(struct.pack("<I", smeta))])
        self.meta(0, mleaf, True)
        struct.pack_into("<I", self.pages[0], 32, len(self.pages) - 1)
        return b"".join(bytes(p) for p in self.pages)


def test_bdb_wallet_dat_is_imported_on_start(tmp_path):
    sec = hashlib.sha256(b"bdb import test key").digest()
    pub = ref.pubkey_from_secret(sec, True)
    addr = b58check(b"\x6f" + hash160(pub))  # regtest P2PKH
    # the reference's "key" record: DER SEC1 ECPrivateKey (version 1, secret, tagged curve
    # parameters, public key) and the trailing hash of pubkey || privkey
    inner = b"\x02\x01\x01\x04\x20" + sec + b"\xa0\x03\x06\x01\x00" + b"\xa1\x24\x03\x22\x00" + pub
    der = b"\x30\x81" + bytes([len(inner)]) + inner
    recs = [
        (ser_bytes(b"key") + ser_bytes(pub), ser_bytes(der) + hashlib.sha256(pub + der).digest()),
        (ser_bytes(b"minversion"), struct.pack("<i", 60000)),
        (ser_bytes(b"orderposnext"), struct.pack("<q", 0)),
    ]
    recs.sort()
    datadir = tmp_path / "n"
    wdir = datadir / "regtest"
    wdir.mkdir(parents=True)
    (wdir / "wallet.dat").write_bytes(BdbWriter().file(recs))
    n = BcpdProcess(str(datadir), extra_args=["-gpu=0"])
    n.start()
    try:
        assert n.rpc.validateaddress(addr)["ismine"] is True
        wif = b58check(b"\xef" + sec + b"\x01")
        assert n.rpc.dumpprivkey(addr) == wif
        assert any(p.startswith("wallet.dat.bdb.") for p in os.listdir(wdir))  # the original, kept
        assert os.path.isdir(wdir / "wallet.dat")  # now this node's store
    finally:
        n.stop()
    log = (wdir / "debug.log").read_text(errors="replace")
    assert "Imported 3 records from the Berkeley DB wallet" in log
