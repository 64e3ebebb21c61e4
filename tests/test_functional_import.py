"""Chain export/import (reference contrib/linearize + init.cpp ThreadImport, -loadblock,
bootstrap.dat): a regtest chain that crosses the BCP fork (legacy 80-byte headers, then
140-byte Equihash(48,5) headers) is listed by linearize-hashes.py over RPC, written in order
to bootstrap.dat by linearize-data.py from the node's blk files, and imported by fresh
nodes through -loadblock and through <datadir>/bootstrap.dat (renamed .old afterwards)."""
import os
import shutil
import subprocess
import sys
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIN = os.path.join(ROOT, "contrib", "linearize")


def wait_height(node, h, timeout=120):
    end = time.time() + timeout
    while time.time() < end:
        if node.rpc.getblockcount() == h:
            return
        time.sleep(0.2)
    raise AssertionError(f"height {node.rpc.getblockcount()} != {h}")


def test_linearize_and_import(tmp_path):
    src = BcpdProcess(str(tmp_path / "src"), extra_args=["-gpu=0"])
    src.start()
    try:
        src.rpc.generate(3004)  # crosses BCPHeight=3000 on regtest
        tip = src.rpc.getbestblockhash()
        cfg = tmp_path / "lin.cfg"
        cfg.write_text(f"port={src.rpcport}\nrpcuser=rt\nrpcpassword=rtpass\n"
                       f"input={tmp_path / 'src' / 'regtest' / 'blocks'}\nhashlist={tmp_path / 'hashes.txt'}\n"
                       f"output_file={tmp_path / 'bootstrap.dat'}\n")
        with open(tmp_path / "hashes.txt", "w") as out:
            subprocess.run([sys.executable, os.path.join(LIN, "linearize-hashes.py"), str(cfg)], stdout=out, check=True)
    finally:
        src.stop()
    hashes = open(tmp_path / "hashes.txt").read().split()
    assert len(hashes) == 3005 and hashes[-1] == tip
    r = subprocess.run([sys.executable, os.path.join(LIN, "linearize-data.py"), str(cfg)], capture_output=True,
                       text=True, check=True)
    assert "3005 blocks" in r.stdout

    # -loadblock
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0", f"-loadblock={tmp_path / 'bootstrap.dat'}"])
    a.start()
    try:
        wait_height(a, 3004)
        assert a.rpc.getbestblockhash() == tip
    finally:
        a.stop()

    # <datadir>/bootstrap.dat, renamed after the import
    bdir = tmp_path / "b" / "regtest"
    os.makedirs(bdir)
    shutil.copy(tmp_path / "bootstrap.dat", bdir / "bootstrap.dat")
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    b.start()
    try:
        wait_height(b, 3004)
        assert b.rpc.getbestblockhash() == tip
    finally:
        b.stop()
    assert os.path.exists(bdir / "bootstrap.dat.old") and not os.path.exists(bdir / "bootstrap.dat")
