"""fundrawtransaction, case by case.

Parity: reference test/functional/fundrawtransaction.py (four nodes connected as there, every
node at -keypool=1 as the reference framework's bitcoin.conf, the same chain shape so balance
checks use the reference's numbers). Cases in the reference's order:
 1. simple test; two coins (2.2, 2.6: inputs unsigned); two outputs
 2. a given VIN worth more than needed: inputs + fee = outputs
 3. no change output (changepos -1) when the change would be below the fee tolerance
 4. an unknown option: -3 "Unexpected key foo"
 5. an invalid change address: -5 "changeAddress must be a valid bitcoin address"
 6. a provided change address and changePosition (out of bounds: -8)
 7. a given VIN smaller than needed, with a non-empty scriptSig that is kept
 8. two given VINs; two VINs and two VOUTs
 9. an unknown VIN: -4 "Insufficient funds"
10. fee of the funded transaction = fee of the same payment by sendtoaddress / sendmany
    (P2PKH, six outputs, 2-of-2 and 4-of-5 P2SH multisig), within 2 bytes per input
11. spending a 2-of-2 multisig output through fundrawtransaction + signrawtransaction
12. locked wallet: funding needs no private key, sending does (-13), signing after unlock
13. ~20 small inputs: fee comparison, then sign and send
14. OP_RETURN output and no VIN: one input and a change output are added
15. watch-only: includeWatching funds from a watched key only; the whole watched amount
    (positional includeWatching = true) needs a second signer
16. feeRate option: 2x / 10x the default rate
17. reserveChangeKey false keeps the change key in the keypool
18. subtractFeeFromOutputs: the fee comes out of the chosen outputs, shares equal
"""
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError("timeout")


def D(x):
    return Decimal(str(x))


def raises(code, msg, fn, *args):
    with pytest.raises(RPCError) as e:
        fn(*args)
    assert e.value.code == code, (e.value.code, str(e.value))
    if msg:
        assert msg in str(e.value), str(e.value)


def get_unspent(listunspent, amount):
    for utx in listunspent:
        if D(utx["amount"]) == D(amount):
            return utx
    raise AssertionError(f"unspent output with amount {amount} not found")


def count_bytes(hexstr):
    return len(bytearray.fromhex(hexstr))


def assert_fee_amount(fee, tx_size, fee_per_kb):
    """Reference test_framework/util.py assert_fee_amount: at least the target, at most two
    bytes' worth above it."""
    target = D(tx_size) * D(fee_per_kb) / 1000
    fee = D(fee)
    assert fee >= target.quantize(D("0.00000001")), (fee, target)
    assert fee <= ((D(tx_size) + 2) * D(fee_per_kb) / 1000).quantize(D("0.00000001")) + D("0.00000001"), (fee, target)


@pytest.fixture
def nodes(tmp_path):
    ns = [BcpdProcess(str(tmp_path / f"n{i}"), extra_args=["-gpu=0", "-keypool=1"]) for i in range(4)]
    for n in ns:
        n.start()
    for a, b in ((0, 1), (1, 2), (0, 2), (0, 3)):
        ns[a].rpc.addnode(f"127.0.0.1:{ns[b].p2p_port}", "onetry")
    # connected = handshake done on both sides (the reference's connect_nodes_bi): a block mined
    # before that is not announced to the peer, which only asks its first peer for headers in IBD
    wait_until(lambda: [n.rpc.getconnectioncount() for n in ns] == [3, 2, 2, 1] and
               all(p["version"] for n in ns for p in n.rpc.getpeerinfo()))
    yield ns
    for n in ns:
        n.stop()


def sync_all(ns):
    try:
        wait_until(lambda: len({n.rpc.getbestblockhash() for n in ns}) == 1)
    except AssertionError:
        raise AssertionError(f"tips differ: {[n.rpc.getblockcount() for n in ns]} "
                             f"peers {[n.rpc.getconnectioncount() for n in ns]}")
    wait_until(lambda: len({tuple(sorted(n.rpc.getrawmempool())) for n in ns}) == 1)


def test_fundrawtransaction(nodes):
    n0, n1, n2, n3 = (n.rpc for n in nodes)
    min_relay_tx_fee = D(n0.getnetworkinfo()["relayfee"])
    for n in (n0, n1, n2, n3):
        n.settxfee(min_relay_tx_fee)
    fee_tolerance = 2 * min_relay_tx_fee / 1000

    n2.generate(1)
    sync_all(nodes)
    n0.generate(121)
    sync_all(nodes)

    watchonly_address = n0.getnewaddress()
    watchonly_pubkey = n0.validateaddress(watchonly_address)["pubkey"]
    watchonly_amount = D(200)
    n3.importpubkey(watchonly_pubkey, "", True)
    watchonly_txid = n0.sendtoaddress(watchonly_address, watchonly_amount)
    n0.sendtoaddress(n3.getnewaddress(), watchonly_amount / 10)
    n0.sendtoaddress(n2.getnewaddress(), 1.5)
    n0.sendtoaddress(n2.getnewaddress(), 1.0)
    n0.sendtoaddress(n2.getnewaddress(), 5.0)
    sync_all(nodes)
    n0.generate(1)
    sync_all(nodes)

    # 1. simple tests
    rawtx = n2.createrawtransaction([], {n0.getnewaddress(): 1.0})
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert len(dec["vin"]) > 0
    rawtx = n2.createrawtransaction([], {n0.getnewaddress(): 2.2})
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert len(dec["vin"]) > 0
    rawtx = n2.createrawtransaction([], {n0.getnewaddress(): 2.6})
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert len(dec["vin"]) > 0 and dec["vin"][0]["scriptSig"]["hex"] == ""
    rawtx = n2.createrawtransaction([], {n0.getnewaddress(): 2.6, n1.getnewaddress(): 2.5})
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert len(dec["vin"]) > 0 and dec["vin"][0]["scriptSig"]["hex"] == ""

    # 2. a VIN worth more than needed
    utx = get_unspent(n2.listunspent(), 5)
    rawtx = n2.createrawtransaction([{"txid": utx["txid"], "vout": utx["vout"]}], {n0.getnewaddress(): 1.0})
    assert n2.decoderawtransaction(rawtx)["vin"][0]["txid"] == utx["txid"]
    fund = n2.fundrawtransaction(rawtx)
    fee = D(fund["fee"])
    dec = n2.decoderawtransaction(fund["hex"])
    assert fee + sum(D(o["value"]) for o in dec["vout"]) == D(utx["amount"])

    # 3. no change output
    utx = get_unspent(n2.listunspent(), 5)
    rawtx = n2.createrawtransaction([{"txid": utx["txid"], "vout": utx["vout"]}],
                                    {n0.getnewaddress(): D(5.0) - fee - fee_tolerance})
    fund = n2.fundrawtransaction(rawtx)
    fee = D(fund["fee"])
    dec = n2.decoderawtransaction(fund["hex"])
    assert fund["changepos"] == -1
    assert fee + sum(D(o["value"]) for o in dec["vout"]) == D(utx["amount"])

    # 4-6. options
    utx = get_unspent(n2.listunspent(), 5)
    rawtx = n2.createrawtransaction([{"txid": utx["txid"], "vout": utx["vout"]}], {n0.getnewaddress(): D(4.0)})
    raises(-3, "Unexpected key foo", n2.fundrawtransaction, rawtx, {"foo": "bar"})
    raises(-5, "changeAddress must be a valid bitcoin address", n2.fundrawtransaction, rawtx,
           {"changeAddress": "foobar"})
    change = n2.getnewaddress()
    raises(-8, "changePosition out of bounds", n2.fundrawtransaction, rawtx,
           {"changeAddress": change, "changePosition": 2})
    fund = n2.fundrawtransaction(rawtx, {"changeAddress": change, "changePosition": 0})
    out = n2.decoderawtransaction(fund["hex"])["vout"][0]
    assert out["scriptPubKey"]["addresses"][0] == change

    # 7. a VIN smaller than needed, whose (non-empty) scriptSig is kept
    utx = get_unspent(n2.listunspent(), 1)
    outputs = {n0.getnewaddress(): 1.0}
    rawtx = n2.createrawtransaction([{"txid": utx["txid"], "vout": utx["vout"]}], outputs)
    rawtx = rawtx[:82] + "0100" + rawtx[84:]  # 4-byte version + 1-byte vin count + 36-byte prevout, script_len
    dec = n2.decoderawtransaction(rawtx)
    assert dec["vin"][0]["txid"] == utx["txid"] and dec["vin"][0]["scriptSig"]["hex"] == "00"
    fund = n2.fundrawtransaction(rawtx)
    dec = n2.decoderawtransaction(fund["hex"])
    matching = 0
    for i, o in enumerate(dec["vout"]):
        if o["scriptPubKey"]["addresses"][0] in outputs:
            matching += 1
        else:
            assert i == fund["changepos"]
    assert dec["vin"][0]["txid"] == utx["txid"] and dec["vin"][0]["scriptSig"]["hex"] == "00"
    assert matching == 1 and len(dec["vout"]) == 2

    # 8. two VINs; two VINs and two VOUTs
    utx = get_unspent(n2.listunspent(), 1)
    utx2 = get_unspent(n2.listunspent(), 5)
    inputs = [{"txid": utx["txid"], "vout": utx["vout"]}, {"txid": utx2["txid"], "vout": utx2["vout"]}]
    outputs = {n0.getnewaddress(): 6.0}
    rawtx = n2.createrawtransaction(inputs, outputs)
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert sum(o["scriptPubKey"]["addresses"][0] in outputs for o in dec["vout"]) == 1 and len(dec["vout"]) == 2
    assert sum(1 for v in dec["vin"] for i in inputs if i["txid"] == v["txid"]) == 2
    outputs = {n0.getnewaddress(): 6.0, n0.getnewaddress(): 1.0}
    rawtx = n2.createrawtransaction(inputs, outputs)
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert sum(o["scriptPubKey"]["addresses"][0] in outputs for o in dec["vout"]) == 2 and len(dec["vout"]) == 3

    # 9. an unknown VIN
    rawtx = n2.createrawtransaction(
        [{"txid": "1c7f966dab21119bac53213a2bc7532bff1fa844c124fd750a7d0b1332440bd1", "vout": 0}],
        {n0.getnewaddress(): 1.0})
    raises(-4, "Insufficient funds", n2.fundrawtransaction, rawtx)
    invalid_vin_tx = rawtx

    # 10. fees equal those of the same payment made by the wallet
    def compare_fee(funded, txid, tolerance=fee_tolerance):
        signed_fee = D(n0.getrawmempool(True)[txid]["fee"]) if txid in n0.getrawmempool() else None
        delta = D(funded["fee"]) - signed_fee
        assert 0 <= delta <= tolerance, (funded["fee"], signed_fee)

    outputs = {n1.getnewaddress(): 1.1}
    funded = n0.fundrawtransaction(n0.createrawtransaction([], outputs))
    compare_fee(funded, n0.sendtoaddress(n1.getnewaddress(), 1.1))
    outputs = {n1.getnewaddress(): v for v in (1.1, 1.2, 0.1, 1.3, 0.2, 0.3)}
    funded = n0.fundrawtransaction(n0.createrawtransaction([], outputs))
    compare_fee(funded, n0.sendmany("", outputs))
    for m, k in ((2, 2), (4, 5)):
        pubs = [n1.validateaddress(n1.getnewaddress())["pubkey"] for _ in range(k)]
        msig = n1.addmultisigaddress(m, pubs)
        funded = n0.fundrawtransaction(n0.createrawtransaction([], {msig: 1.1}))
        compare_fee(funded, n0.sendtoaddress(msig, 1.1))

    # 11. spend a 2-of-2 multisig output over fundrawtransaction
    pubs = [n2.validateaddress(n2.getnewaddress())["pubkey"] for _ in range(2)]
    msig = n2.addmultisigaddress(2, pubs)
    n0.sendtoaddress(msig, 1.2)
    sync_all(nodes)
    n1.generate(1)
    sync_all(nodes)
    old_balance = D(n1.getbalance())
    funded = n2.fundrawtransaction(n2.createrawtransaction([], {n1.getnewaddress(): 1.1}))
    signed = n2.signrawtransaction(funded["hex"], None, None, "ALL|FORKID")
    n2.sendrawtransaction(signed["hex"])
    sync_all(nodes)
    n1.generate(1)
    sync_all(nodes)
    assert D(n1.getbalance()) == old_balance + D("1.10000000")

    # 12. locked wallet
    n1.encryptwallet("test")
    if nodes[1].proc.poll() is not None or not _rpc_up(nodes[1]):  # (a node that stops after encryption)
        nodes[1].start()
        nodes[1].rpc.addnode(f"127.0.0.1:{nodes[2].p2p_port}", "onetry")
        nodes[0].rpc.addnode(f"127.0.0.1:{nodes[1].p2p_port}", "onetry")
        n1 = nodes[1].rpc
        n1.settxfee(min_relay_tx_fee)
    n1.getnewaddress()  # drain the keypool
    # (the reference passes the unknown-VIN transaction here, hence "Insufficient funds")
    raises(-4, "Insufficient funds", n1.fundrawtransaction, invalid_vin_tx)
    n1.walletpassphrase("test", 100)  # refills the keypool
    n1.walletlock()
    raises(-13, "walletpassphrase", n1.sendtoaddress, n0.getnewaddress(), 1.2)
    old_balance = D(n0.getbalance())
    funded = n1.fundrawtransaction(n1.createrawtransaction([], {n0.getnewaddress(): 1.1}))  # no key needed
    n1.walletpassphrase("test", 600)
    signed = n1.signrawtransaction(funded["hex"], None, None, "ALL|FORKID")
    n1.sendrawtransaction(signed["hex"])
    n1.generate(1)
    sync_all(nodes)
    assert D(n0.getbalance()) == old_balance + D("51.10000000")  # 1.1 + a coinbase of node 0 maturing

    # 13. ~20 small inputs: fee comparison, then sign and send
    n1.sendtoaddress(n0.getnewaddress(), n1.getbalance(), "", "", True)
    sync_all(nodes)
    n0.generate(1)
    sync_all(nodes)
    for _ in range(20):
        n0.sendtoaddress(n1.getnewaddress(), 0.01)
    n0.generate(1)
    sync_all(nodes)
    outputs = {n0.getnewaddress(): 0.15, n0.getnewaddress(): 0.04}
    funded = n1.fundrawtransaction(n1.createrawtransaction([], outputs))
    txid = n1.sendmany("", outputs)
    delta = D(funded["fee"]) - D(n1.getrawmempool(True)[txid]["fee"])
    assert 0 <= delta <= fee_tolerance * 19
    n1.sendtoaddress(n0.getnewaddress(), n1.getbalance(), "", "", True)
    sync_all(nodes)
    n0.generate(1)
    sync_all(nodes)
    for _ in range(20):
        n0.sendtoaddress(n1.getnewaddress(), 0.01)
    n0.generate(1)
    sync_all(nodes)
    old_balance = D(n0.getbalance())
    funded = n1.fundrawtransaction(n1.createrawtransaction([], {n0.getnewaddress(): 0.15, n0.getnewaddress(): 0.04}))
    signed = n1.signrawtransaction(funded["hex"], None, None, "ALL|FORKID")
    n1.sendrawtransaction(signed["hex"])
    sync_all(nodes)
    n0.generate(1)
    sync_all(nodes)
    assert D(n0.getbalance()) == old_balance + D("50.19000000")  # 0.19 + block reward

    # 14. OP_RETURN output and no VIN
    rawtx = "0100000000010000000000000000066a047465737400000000"
    dec = n2.decoderawtransaction(rawtx)
    assert len(dec["vin"]) == 0 and len(dec["vout"]) == 1
    dec = n2.decoderawtransaction(n2.fundrawtransaction(rawtx)["hex"])
    assert len(dec["vin"]) > 0 and len(dec["vout"]) == 2

    # 15. watch-only funds
    rawtx = n3.createrawtransaction([], {n2.getnewaddress(): watchonly_amount / 2})
    result = n3.fundrawtransaction(rawtx, {"includeWatching": True})
    res = n0.decoderawtransaction(result["hex"])
    assert len(res["vin"]) == 1 and res["vin"][0]["txid"] == watchonly_txid
    assert "fee" in result and result["changepos"] > -1
    rawtx = n3.createrawtransaction([], {n2.getnewaddress(): watchonly_amount})
    result = n3.fundrawtransaction(rawtx, True)  # positional includeWatching (backward compatibility)
    res = n0.decoderawtransaction(result["hex"])
    assert len(res["vin"]) == 2 and watchonly_txid in (res["vin"][0]["txid"], res["vin"][1]["txid"])
    assert D(result["fee"]) > 0 and result["changepos"] > -1
    assert D(result["fee"]) + D(res["vout"][result["changepos"]]["value"]) == watchonly_amount / 10
    signed = n3.signrawtransaction(result["hex"], None, None, "ALL|FORKID")
    assert not signed["complete"]
    signed = n0.signrawtransaction(signed["hex"], None, None, "ALL|FORKID")
    assert signed["complete"]
    n0.sendrawtransaction(signed["hex"])
    n0.generate(1)
    sync_all(nodes)

    # 16. feeRate
    assert len(n3.listunspent(1)) == 1  # one input, so coin selection cannot skew the result
    rawtx = n3.createrawtransaction([], {n3.getnewaddress(): 1})
    result = n3.fundrawtransaction(rawtx)
    result2 = n3.fundrawtransaction(rawtx, {"feeRate": 2 * min_relay_tx_fee})
    result3 = n3.fundrawtransaction(rawtx, {"feeRate": 10 * min_relay_tx_fee})
    rate = D(result["fee"]) * 1000 / count_bytes(result["hex"])
    assert_fee_amount(result2["fee"], count_bytes(result2["hex"]), 2 * rate)
    assert_fee_amount(result3["fee"], count_bytes(result3["hex"]), 10 * rate)

    # 17. reserveChangeKey
    def change_address(res_hex):
        return "".join(o["scriptPubKey"]["addresses"][0] for o in n0.decoderawtransaction(res_hex)["vout"]
                       if D(o["value"]) > 1)

    ca = change_address(n3.fundrawtransaction(rawtx, {"reserveChangeKey": False})["hex"])
    assert ca and ca == n3.getnewaddress()  # the key stayed in the keypool
    ca = change_address(n3.fundrawtransaction(rawtx)["hex"])
    assert ca and ca != n3.getnewaddress()  # now it is taken

    # 18. subtractFeeFromOutputs
    assert len(n3.listunspent(1)) == 1
    rawtx = n3.createrawtransaction([], {n2.getnewaddress(): 1})
    result = [n3.fundrawtransaction(rawtx), n3.fundrawtransaction(rawtx, {"subtractFeeFromOutputs": []}),
              n3.fundrawtransaction(rawtx, {"subtractFeeFromOutputs": [0]}),
              n3.fundrawtransaction(rawtx, {"feeRate": 2 * min_relay_tx_fee}),
              n3.fundrawtransaction(rawtx, {"feeRate": 2 * min_relay_tx_fee, "subtractFeeFromOutputs": [0]})]
    dec = [n3.decoderawtransaction(r["hex"]) for r in result]
    output = [D(d["vout"][1 - r["changepos"]]["value"]) for d, r in zip(dec, result)]
    change = [D(d["vout"][r["changepos"]]["value"]) for d, r in zip(dec, result)]
    fees = [D(r["fee"]) for r in result]
    assert fees[0] == fees[1] == fees[2] and fees[3] == fees[4]
    assert change[0] == change[1] and output[0] == output[1]
    assert output[0] == output[2] + fees[2] and change[0] + fees[0] == change[2]
    assert output[3] == output[4] + fees[4] and change[3] + fees[3] == change[4]
    outputs = {n2.getnewaddress(): v for v in (1.0, 1.1, 1.2, 1.3)}
    rawtx = n3.createrawtransaction([], outputs)
    result = [n3.fundrawtransaction(rawtx), n3.fundrawtransaction(rawtx, {"subtractFeeFromOutputs": [0, 2, 3]})]
    dec = [n3.decoderawtransaction(r["hex"]) for r in result]
    output = [[D(o["value"]) for i, o in enumerate(d["vout"]) if i != r["changepos"]] for d, r in zip(dec, result)]
    share = [a - b for a, b in zip(output[0], output[1])]
    assert share[1] == 0 and share[0] > 0 and share[2] > 0 and share[3] > 0
    assert share[2] == share[3]  # outputs 2 and 3 take the same share of the fee


def _rpc_up(n):
    try:
        n.rpc.getblockcount()
        return True
    except Exception:
        return False
