"""-salvagewallet (reference qa/rpc-tests via CWalletDB::Recover / CDBEnv::Salvage): a wallet
whose store log has a damaged record in the middle still loads its keys after a restart with
-salvagewallet — the damaged stretch is skipped, later intact batches are kept, the original
store is moved aside as a .bak, and the implied rescan restores the balance."""
import glob
import os
import struct
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.process import BcpdProcess

pytestmark = pytest.mark.functional

BATCH_MAGIC = struct.pack("<I", 0xB7C0DB02)  # write-ahead log record header (csrc/node/kvstore.cpp)


def test_salvagewallet_recovers_keys(tmp_path):
    d = str(tmp_path / "s")
    n = BcpdProcess(d, extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        n.rpc.generate(101)
        early = n.rpc.getnewaddress()
        early_priv = n.rpc.dumpprivkey(early)
        filler = [n.rpc.getnewaddress() for _ in range(3)]
        late = n.rpc.getnewaddress()
        late_priv = n.rpc.dumpprivkey(late)
        bal = Decimal(str(n.rpc.getbalance()))
        port = n.rpcport
    finally:
        n.stop()
    logs = [p for p in glob.glob(os.path.join(d, "**", "kv-*.log"), recursive=True)
            if "wallet.dat" in p and os.path.getsize(p) > 0]
    assert len(logs) == 1
    data = bytearray(open(logs[0], "rb").read())
    # damage the payload of a batch in the middle of the log (CRC now fails for it)
    starts = [i for i in range(len(data) - 3) if data[i:i + 4] == BATCH_MAGIC]
    victim = starts[len(starts) // 2]
    for i in range(victim + 12, min(victim + 20, len(data))):
        data[i] ^= 0xFF
    open(logs[0], "wb").write(bytes(data))

    n2 = BcpdProcess(d, extra_args=["-gpu=0", "-keypool=5", "-salvagewallet"], port=port)
    n2.start()
    try:
        assert n2.rpc.dumpprivkey(early) == early_priv
        assert n2.rpc.dumpprivkey(late) == late_priv
        assert Decimal(str(n2.rpc.getbalance())) == bal
        assert filler
    finally:
        n2.stop()
    wallet_dir = os.path.dirname(logs[0])
    assert glob.glob(wallet_dir + ".*.bak")
