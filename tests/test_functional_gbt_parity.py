"""getblocktemplate parity with the reference's BIP22/BIP23/BIP9 handler.

Parity: reference src/rpc/mining.cpp:428-897 (getblocktemplate) and
test/functional/getblocktemplate_proposals.py:
* a lone node refuses templates with RPC_CLIENT_NOT_CONNECTED (-9) "Bitcoin is not connected!";
  a node in initial block download with RPC_CLIENT_IN_INITIAL_DOWNLOAD (-10), regtest included
  (:643-656);
* proposals: "duplicate" for a known block, "inconclusive-not-best-prevblk" for a stale parent,
  "inconclusive-bad-height" when the header's height is not tip+1 (:564-616); the
  `proposal_legacy` mode decodes an 80-byte-header block, which carries no height, so a new
  legacy block always ends at the height check (:611-616, the unconditional second check);
* a pre-versionbits client (`maxversion` and no `rules`) gets "version/force" among the mutable
  fields (:631-634, :856-865); a versionbits client does not;
* sizelimit / sigoplimit are the default 8 MB limits whatever -excessiveblocksize is (:882-885);
* mode errors: an unknown mode (-8 "Invalid mode"), a proposal without data (-3).
The "requires explicit client support" error (:837-845) needs an active deployment without
gbt_force; the reference's deployments (testdummy, csv) are all gbt_force, so it is unreachable
there as here.
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase
from bitcoincashplus_amd.testing.messages import CBlock, CTransaction, from_hex

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

MAX_BLOCK_SIZE = 8_000_000
MAX_SIGOPS = 20_000 * 8  # GetMaxBlockSigOpsCount(8 MB): 20k per started megabyte


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError("timed out")


def rpc_error(fn, *args):
    with pytest.raises(RPCError) as e:
        fn(*args)
    return e.value


@pytest.fixture
def pair(tmp_path):
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0", "-excessiveblocksize=16000000"])
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    a.start()
    b.start()
    yield a, b
    a.stop()
    b.stop()


def test_refusals_lone_node_and_ibd(pair):
    a, b = pair
    # fresh regtest chain (genesis only, 2011 timestamp): still in initial block download
    e = rpc_error(a.rpc.getblocktemplate)
    assert e.code == -9 and "Bitcoin is not connected!" in str(e)  # no peers is checked first
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() == 1 and b.rpc.getconnectioncount() == 1)
    e = rpc_error(a.rpc.getblocktemplate)
    assert e.code == -10 and "Bitcoin is downloading blocks..." in str(e)
    a.rpc.generate(101)  # a recent tip ends IBD
    wait_until(lambda: b.rpc.getblockcount() == 101)
    tmpl = a.rpc.getblocktemplate()
    assert tmpl["height"] == 102
    # the peer leaves: refused again
    for p in a.rpc.getpeerinfo():
        a.rpc.disconnectnode(p["addr"])
    wait_until(lambda: a.rpc.getconnectioncount() == 0)
    e = rpc_error(a.rpc.getblocktemplate)
    assert e.code == -9


def test_template_fields_and_proposals(pair):
    a, b = pair
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() == 1)
    a.rpc.generate(110)
    wait_until(lambda: b.rpc.getblockcount() == 110)

    tmpl = a.rpc.getblocktemplate()
    # default limits, not the node's -excessiveblocksize
    assert tmpl["sizelimit"] == MAX_BLOCK_SIZE and tmpl["sigoplimit"] == MAX_SIGOPS
    assert tmpl["mutable"] == ["time", "transactions", "prevblock"]
    assert not any(r.startswith("!") for r in tmpl["rules"]) and not any(k.startswith("!") for k in tmpl["vbavailable"])
    # maxversion from a pre-versionbits client: version/force; ignored next to a rules array
    assert "version/force" in a.rpc.getblocktemplate({"maxversion": 4})["mutable"]
    assert "version/force" not in a.rpc.getblocktemplate({"maxversion": 1})["mutable"]
    assert "version/force" not in a.rpc.getblocktemplate({"rules": [], "maxversion": 4})["mutable"]

    # mode errors
    e = rpc_error(a.rpc.getblocktemplate, {"mode": "nosuchmode"})
    assert e.code == -8 and "Invalid mode" in str(e)
    e = rpc_error(a.rpc.getblocktemplate, {"mode": "proposal"})
    assert e.code == -3 and "Missing data String key for proposal" in str(e)
    e = rpc_error(a.rpc.getblocktemplate, {"mode": "proposal_legacy", "data": "00"})
    assert e.code == -22

    # proposals
    height = tmpl["height"]
    cb = create_coinbase(height)
    cb.vout[0].nValue = tmpl["coinbasevalue"]
    cb.rehash()
    txs = [from_hex(CTransaction(), t["data"]) for t in tmpl["transactions"]]
    prev = int(tmpl["previousblockhash"], 16)

    def block(h=height, parent=prev):
        return create_block(parent, cb, tmpl["curtime"], h, int(tmpl["bits"], 16), tmpl["version"], txs)

    good = block()
    assert a.rpc.getblocktemplate({"mode": "proposal", "data": good.serialize().hex()}) is None
    # the header's height must be tip + 1
    assert a.rpc.getblocktemplate({"mode": "proposal", "data": block(h=height + 1).serialize().hex()}) == \
        "inconclusive-bad-height"
    assert a.rpc.getblocktemplate({"mode": "proposal", "data": block(h=height - 1).serialize().hex()}) == \
        "inconclusive-bad-height"
    # legacy format (80-byte header, no height): decodes, then always fails the height check
    assert a.rpc.getblocktemplate({"mode": "proposal_legacy", "data": good.serialize(legacy=True).hex()}) == \
        "inconclusive-bad-height"
    # a stale parent is checked before the height
    stale = block(h=5, parent=int(a.rpc.getblockhash(4), 16))
    assert a.rpc.getblocktemplate({"mode": "proposal_legacy", "data": stale.serialize(legacy=True).hex()}) == \
        "inconclusive-not-best-prevblk"
    # known blocks: duplicate, in either encoding
    tip_hex = a.rpc.getblock(a.rpc.getbestblockhash(), False)
    assert a.rpc.getblocktemplate({"mode": "proposal", "data": tip_hex}) == "duplicate"
    tip_blk = from_hex(CBlock(), tip_hex)
    assert a.rpc.getblocktemplate({"mode": "proposal_legacy", "data": tip_blk.serialize(legacy=True).hex()}) == \
        "duplicate"
