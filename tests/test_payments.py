"""BIP70 payment protocol (csrc/wallet/paymentrequest.{h,cpp}, RPC decodepaymentrequest /
sendpaymentrequest).

Parity: reference src/qt/test/paymentservertests.cpp. That test feeds the payment requests of
src/qt/test/paymentrequestdata.h through PaymentServer and checks the authenticated merchant,
verifyNetwork, verifyExpired, verifySize and verifyAmount; `test_reference_vectors` runs the same
checks on the same vectors (read from the reference tree when it is mounted). The reference
verifies certificates at the current time, and its fixture certificates expired in 2022, so
here the verification time is pinned to 2017-01-01, when every fixture certificate the reference
expects to pass was valid. The self-contained tests build their own CA, merchant certificate and
signed requests with the openssl CLI.
"""
import base64
import os
import json
import re
import shutil
import subprocess

import pytest

from bitcoincashplus_amd import native

REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "vectors", "paymentrequest_vectors.json")
T2017 = 1483228800


def _ref_vectors():
    # the reference's BIP70 test payloads (src/qt/test/paymentrequestdata.h), vendored as JSON
    with open(REF_DATA) as f:
        return {k: base64.b64decode(v) for k, v in json.load(f)["vectors"].items()}


def test_reference_vectors():
    v = _ref_vectors()
    ca1, ca2 = [v["caCert1"]], [v["caCert2"]]

    def merchant(name, roots):
        info = native.payment_request_info(v[name], roots, "main", T2017)
        assert info["initialized"]
        return info["merchant"]

    assert merchant("paymentrequest1_cert1", ca1) == "testmerchant.org"  # direct to caCert1
    assert merchant("paymentrequest2_cert1", ca1) == ""                  # expired merchant cert
    assert merchant("paymentrequest3_cert1", ca1) == "testmerchant8.org"  # 10-long chain
    assert merchant("paymentrequest4_cert1", ca1) == ""                  # expired intermediate
    assert merchant("paymentrequest5_cert1", ca1) == ""                  # CA not in the root list
    assert merchant("paymentrequest1_cert1", []) == ""                   # no roots at all

    def info(name):
        i = native.payment_request_info(v[name], ca2, "main", T2017)
        assert i["initialized"]
        # proto2 re-serialization is byte-exact (what a signature covers)
        assert i["reserialized"] == v[name]
        return i

    assert info("paymentrequest1_cert2")["network_ok"] is False   # testnet request, main client
    assert info("paymentrequest2_cert2")["expired"] is True       # expires = 1
    assert info("paymentrequest3_cert2")["expired"] is False      # expires = 2^63 - 1
    assert info("paymentrequest4_cert2")["expired"] is True       # expires = 2^63 (negative as int64)
    outs = info("paymentrequest5_cert2")["outputs"]               # 21,000,001 coins
    assert outs and all(ok is False for _, _, ok in outs)


def test_size_limit_and_garbage():
    big = os.urandom(native.BIP70_MAX_PAYMENTREQUEST_SIZE + 1)
    i = native.payment_request_info(big)
    assert i["size_ok"] is False
    assert i["initialized"] is False
    # missing the required serialized_payment_details
    assert native.payment_request_info(b"\x12\x04none")["initialized"] is False
    # truncated length prefix
    assert native.payment_request_info(b"\x22\x10ab")["initialized"] is False
    # up-version payment details are refused
    req = native.payment_request_build([(1000, b"\x51")], 1, version=2)
    assert native.payment_request_info(req)["initialized"] is False


def test_build_roundtrip_and_checks():
    script = bytes.fromhex("76a914" + "11" * 20 + "88ac")
    req = native.payment_request_build([(12345, script), (2**63, script)], 1700000000, expires=1700000600,
                                       network="regtest", memo="order 7", payment_url="http://m/pay",
                                       merchant_data=b"\x01\x02")
    i = native.payment_request_info(req, [], "regtest", 1700000100)
    assert i["initialized"] and i["pki_type"] == "none" and i["merchant"] == ""
    assert "pki_type == none" in i["merchant_error"]
    assert i["network_ok"] and not i["expired"]
    assert native.payment_request_info(req, [], "regtest", 1700000601)["expired"]
    assert native.payment_request_info(req, [], "main", 1700000100)["network_ok"] is False
    assert i["memo"] == "order 7" and i["payment_url"] == "http://m/pay" and i["merchant_data"] == b"\x01\x02"
    assert i["outputs"][0] == (script, 12345, True)
    assert i["outputs"][1][2] is False  # 2^63 satoshis is out of range
    assert i["reserialized"] == req


def _openssl(*args, **kw):
    subprocess.run(["openssl", *args], check=True, capture_output=True, **kw)


@pytest.fixture
def pki(tmp_path):
    if not shutil.which("openssl"):
        pytest.skip("openssl CLI not available")
    d = tmp_path
    # root CA, intermediate, merchant (RSA 2048, SHA-256)
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", d / "ca.key", "-out", d / "ca.pem",
             "-days", "3650", "-subj", "/CN=Test Root CA")
    ext = d / "ext.cnf"
    ext.write_text("[v3_ca]\nbasicConstraints=critical,CA:TRUE\nkeyUsage=keyCertSign,cRLSign\n")
    _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", d / "int.key", "-out", d / "int.csr",
             "-subj", "/CN=Test Intermediate")
    _openssl("x509", "-req", "-in", d / "int.csr", "-CA", d / "ca.pem", "-CAkey", d / "ca.key",
             "-CAcreateserial", "-out", d / "int.pem", "-days", "3650", "-extfile", ext, "-extensions", "v3_ca")
    _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", d / "m.key", "-out", d / "m.csr",
             "-subj", "/CN=shop.example")
    _openssl("x509", "-req", "-in", d / "m.csr", "-CA", d / "int.pem", "-CAkey", d / "int.key",
             "-CAcreateserial", "-out", d / "m.pem", "-days", "3650")

    def der(name):
        return subprocess.run(["openssl", "x509", "-in", d / name, "-outform", "DER"], check=True,
                              capture_output=True).stdout

    def sign(data, key="m.key", alg="-sha256"):
        (d / "data.bin").write_bytes(data)
        return subprocess.run(["openssl", "dgst", alg, "-sign", d / key, d / "data.bin"], check=True,
                              capture_output=True).stdout

    return {"dir": d, "ca": der("ca.pem"), "int": der("int.pem"), "m": der("m.pem"), "sign": sign}


def _signed_request(pki, chain, pki_type="x509+sha256", alg="-sha256", key="m.key", network="regtest",
                    outputs=None, expires=None):
    script = bytes.fromhex("76a914" + "22" * 20 + "88ac")
    req = native.payment_request_build(outputs or [(50_000, script)], 1700000000, expires=expires,
                                       network=network, memo="invoice", pki_type=pki_type, chain=chain)
    sig = pki["sign"](native.payment_request_signing_data(req), key=key, alg=alg)
    return native.payment_request_set_signature(req, sig)


def test_merchant_authentication(pki):
    now = 0  # current time: the generated certificates are valid now
    chain = [pki["m"], pki["int"]]
    req = _signed_request(pki, chain)
    i = native.payment_request_info(req, [pki["ca"]], "regtest", now)
    assert i["merchant"] == "shop.example", i["merchant_error"]
    # SHA-1 variant
    req1 = _signed_request(pki, chain, pki_type="x509+sha1", alg="-sha1")
    assert native.payment_request_info(req1, [pki["ca"]], "regtest", now)["merchant"] == "shop.example"
    # untrusted root
    i = native.payment_request_info(req, [], "regtest", now)
    assert i["merchant"] == "" and i["merchant_error"].startswith("SSL error")
    # missing intermediate
    req2 = _signed_request(pki, [pki["m"]])
    assert native.payment_request_info(req2, [pki["ca"]], "regtest", now)["merchant"] == ""
    # signed by the wrong key
    req3 = _signed_request(pki, chain, key="int.key")
    i = native.payment_request_info(req3, [pki["ca"]], "regtest", now)
    assert i["merchant"] == "" and "Bad signature" in i["merchant_error"]
    # tampered details after signing: flip one byte inside serialized_payment_details
    bad = bytearray(req)
    pos = bytes(req).find(b"invoice")
    bad[pos] ^= 0x20
    i = native.payment_request_info(bytes(bad), [pki["ca"]], "regtest", now)
    assert i["initialized"] and i["merchant"] == ""
    # unknown pki type
    req4 = _signed_request(pki, chain, pki_type="x509+md5")
    assert "unknown pki_type" in native.payment_request_info(req4, [pki["ca"]], "regtest", now)["merchant_error"]
    # a self-signed merchant certificate passes only with allow_self_signed
    req5 = _signed_request(pki, [pki["ca"]], key="ca.key")
    assert native.payment_request_info(req5, [], "regtest", now)["merchant"] == ""
    assert native.payment_request_info(req5, [], "regtest", now, True)["merchant"] == "Test Root CA"
    # before the certificates' validity window
    assert native.payment_request_info(req, [pki["ca"]], "regtest", 946684800)["merchant"] == ""


def test_payment_and_ack_roundtrip():
    p = native.payment_ack_roundtrip(b"\x0a\x02md\x12\x03tx1\x1a\x05\x12\x03\x76\xa9\x14\x22\x02hi", "thanks")
    ack, payment, memo = p
    assert memo == "thanks"
    d = native.payment_decode(payment)
    assert d["merchant_data"] == b"md" and d["transactions"] == [b"tx1"] and d["memo"] == "hi"
    assert d["refund_to"] == [(0, b"\x76\xa9\x14")]


@pytest.mark.functional
def test_rpc_decode_and_pay(pki, tmp_path):
    from bitcoincashplus_amd.node.embedded import RPCError
    from bitcoincashplus_amd.node.process import BcpdProcess

    (tmp_path / "roots.pem").write_bytes((pki["dir"] / "ca.pem").read_bytes())
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-keypool=5",
                                                    f"-rootcertificates={tmp_path / 'roots.pem'}"])
    n.start()
    try:
        n.rpc.generate(101)
        merchant_addr = n.rpc.getnewaddress()
        script = bytes.fromhex(n.rpc.validateaddress(merchant_addr)["scriptPubKey"])
        req = _signed_request(pki, [pki["m"], pki["int"]], outputs=[(12_345_678, script)])
        info = n.rpc.decodepaymentrequest(req.hex())
        assert info["merchant"] == "shop.example"
        assert info["network_ok"] and not info["expired"] and info["total_ok"]
        assert info["outputs"][0]["address"] == merchant_addr
        # base64 input works too
        assert n.rpc.decodepaymentrequest(base64.b64encode(req).decode())["merchant"] == "shop.example"
        res = n.rpc.sendpaymentrequest(req.hex(), "paid")
        tx = n.rpc.gettransaction(res["txid"])
        assert any(abs(float(d["amount"]) - 0.12345678) < 1e-9 for d in tx["details"])
        pay = native.payment_decode(bytes.fromhex(res["payment"]))
        assert len(pay["transactions"]) == 1 and pay["memo"] == "paid" and len(pay["refund_to"]) == 1
        assert res["merchant"] == "shop.example"
        # network mismatch and expiry are refused
        wrong = _signed_request(pki, [pki["m"], pki["int"]], network="main", outputs=[(100_000, script)])
        with pytest.raises(RPCError):
            n.rpc.sendpaymentrequest(wrong.hex())
        old = _signed_request(pki, [pki["m"], pki["int"]], outputs=[(100_000, script)], expires=1)
        with pytest.raises(RPCError):
            n.rpc.sendpaymentrequest(old.hex())
        # dust
        dust = _signed_request(pki, [pki["m"], pki["int"]], outputs=[(1, script)])
        with pytest.raises(RPCError):
            n.rpc.sendpaymentrequest(dust.hex())
    finally:
        n.stop()
