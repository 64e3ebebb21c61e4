"""UI signal bus (reference src/ui_interface.h:24, src/noui.cpp): block/header tip
notifications fire as the chain advances, init messages and message boxes reach their
slots, and -blocknotify / -alertnotify style hooks run from NotifyBlockTip."""
import os
import time

import pytest

from bitcoincashplus_amd._native import native
from bitcoincashplus_amd.node.embedded import EmbeddedNode
from bitcoincashplus_amd.node.process import BcpdProcess, BIN_DIR


def test_embedded_node_emits_tip_signals(tmp_path):
    native.ui_track_start()
    try:
        with EmbeddedNode("regtest", str(tmp_path), memory=True, gpu=False) as n:
            n.generate(5)
            native.ui_init_message("hello")
            assert native.ui_init_error("boom") is False
            c = native.ui_track_counts()
    finally:
        native.ui_track_stop()
    assert c["NotifyBlockTip"] == 6 and c["lastTipHeight"] == 5  # genesis + 5
    assert c["NotifyHeaderTip"] >= 1 and c["lastHeaderHeight"] == 5
    assert "hello" in c["initMessages"]
    assert c["ThreadSafeMessageBox"] == 1


def test_disconnected_slots_stop_firing(tmp_path):
    native.ui_track_start()
    native.ui_track_stop()
    with EmbeddedNode("regtest", str(tmp_path), memory=True, gpu=False) as n:
        n.generate(2)
    assert "NotifyBlockTip" not in native.ui_track_counts()


@pytest.mark.skipif(not os.path.exists(os.path.join(BIN_DIR, "bcpd")), reason="bcpd not built")
def test_blocknotify_runs_command(tmp_path):
    out = tmp_path / "notify.txt"
    n = BcpdProcess(str(tmp_path / "n0"), extra_args=["-gpu=0", f"-blocknotify=echo %s >> {out}"])
    with n:
        hashes = n.rpc.generate(3)
        deadline = time.time() + 20
        while time.time() < deadline:
            if out.exists() and len(out.read_text().split()) >= 3:
                break
            time.sleep(0.1)
    got = out.read_text().split()
    assert sorted(got) == sorted(hashes)
