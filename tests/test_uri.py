"""BIP21 payment URIs (csrc/wallet/bitcoinuri.{h,cpp}, RPC parsebitcoinuri / formatbitcoinuri).

Parity: reference src/qt/test/uritests.cpp (uriTestsBase58, uriTestsCashAddr, uriTestFormatURI)
— the same URIs and expected fields, with the main-chain scheme "bitcoincashplus".
"""
import pytest

from bitcoincashplus_amd import native

SCHEME = "bitcoincashplus"
B58 = "175tWpb8K1S7NmH4Zx6rewF9WQrcZv245W"
CASH = "qqqprqq976hvnqkeajpc33u5rt92xw5vm5ylgfku0f"


def parse(uri):
    ok, addr, amount, label, message, r = native.parse_bitcoin_uri(SCHEME, uri)
    return ok, addr, amount, label, message


@pytest.mark.parametrize("addr,expect", [(B58, B58), (CASH, f"{SCHEME}:{CASH}")])
def test_reference_uris(addr, expect):
    if addr == B58:  # no scheme at all
        assert not parse(f"{addr}?req-dontexist=")[0]
    assert not parse(f"{SCHEME}:{addr}?req-dontexist=")[0]
    assert parse(f"{SCHEME}:{addr}?dontexist=") == (True, expect, 0, "", "")
    assert parse(f"{SCHEME}:{addr}?label=Wikipedia Example Address") == (True, expect, 0, "Wikipedia Example Address", "")
    assert parse(f"{SCHEME}:{addr}?amount=0.001")[2] == 100000
    assert parse(f"{SCHEME}:{addr}?amount=1.001")[2] == 100100000
    ok, a, amt, label, _ = parse(f"{SCHEME}:{addr}?amount=100&label=Wikipedia Example")
    assert ok and a == expect and amt == 10000000000 and label == "Wikipedia Example"
    ok, a, _, label, msg = parse(f"{SCHEME}:{addr}?message=Wikipedia Example Address")
    assert ok and a == expect and label == "" and msg == "Wikipedia Example Address"
    ok, a, _, label, _ = parse(f"{SCHEME}://{addr}?message=Wikipedia Example Address")
    assert ok and a == expect and label == ""
    assert parse(f"{SCHEME}:{addr}?req-message=Wikipedia Example Address")[0]
    assert not parse(f"{SCHEME}:{addr}?amount=1,000&label=Wikipedia Example")[0]
    assert not parse(f"{SCHEME}:{addr}?amount=1,000.0&label=Wikipedia Example")[0]


def test_uri_details():
    assert not parse(f"bitcoin:{B58}")[0]                     # wrong scheme
    assert parse(f"BitcoinCashPlus:{B58}")[0]                  # schemes are case-insensitive
    assert parse(f"{SCHEME}:{B58}/")[1] == B58                 # trailing slash from an OS handler
    assert parse(f"{SCHEME}:{B58}?label=a%20b%26c")[3] == "a b&c"
    assert not parse(f"{SCHEME}:{B58}?amount=0.123456789")[0]  # more than 8 decimals
    assert parse(f"{SCHEME}:{B58}?amount=")[2] == 0
    assert native.parse_bitcoin_uri(SCHEME, f"{SCHEME}:{B58}?r=https://m.example/req")[5] == "https://m.example/req"
    assert native.parse_coin_amount("21000000") == 21000000 * 10**8
    assert native.parse_coin_amount("1 000.5") == 100050000000
    assert native.parse_coin_amount("99999999999.00000000") is None  # > 18 digits: beyond 63 bits
    assert native.parse_coin_amount("-1") is None


def test_format_uri():
    assert native.format_bitcoin_uri(f"{SCHEME}:{CASH}", message="test") == f"{SCHEME}:{CASH}?message=test"
    assert native.format_bitcoin_uri("CGXa8qa2kKjkmAYjHFsS5j6y4KNbKfNfUS", message="test", use_cashaddr=False) == \
        f"{SCHEME}:CGXa8qa2kKjkmAYjHFsS5j6y4KNbKfNfUS?message=test"
    uri = native.format_bitcoin_uri(f"{SCHEME}:{CASH}", 100100000, "shop & co", "order 5")
    assert uri == f"{SCHEME}:{CASH}?amount=1.001&label=shop%20%26%20co&message=order%205"
    assert parse(uri) == (True, f"{SCHEME}:{CASH}", 100100000, "shop & co", "order 5")


@pytest.mark.functional
def test_uri_rpcs(tmp_path):
    from bitcoincashplus_amd.node.process import BcpdProcess

    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        addr = n.rpc.getnewaddress()  # Base58 by default (reference src/init.cpp:2119-2120)
        uri = n.rpc.formatbitcoinuri(addr, 1.5, "me", "for coffee")
        # a Base58 address takes the "bitcoincashplus:" scheme (reference src/qt/guiutil.cpp:168-176,263)
        assert uri.startswith(f"bitcoincashplus:{addr}?amount=1.5&label=me&message=for%20coffee")
        r = n.rpc.parsebitcoinuri(uri)
        assert r["address"] == addr and r["isvalid"] and float(r["amount"]) == 1.5
        assert r["label"] == "me" and r["message"] == "for coffee"
    finally:
        n.stop()


def test_address_entry_validator():
    """reference bitcoinaddressvalidatortests.cpp inputTests"""
    v = native.validate_address_input
    assert v("")[0] == "intermediate"
    for ok in ("BIIC", "BITCOINCASHH", "BITC", "BITCOINCASHPLUS:QP", "bitcoincashplus:qp", "bItCoInCaShPlUs:Qp",
               "BBBBBBBBBBBBBB"):
        assert v(ok)[0] == "acceptable", ok
    assert v("%")[0] == "invalid"
    # whitespace and zero-width spaces are stripped, not rejected
    assert v(" bitcoincashplus:​qp \t﻿") == ("acceptable", "bitcoincashplus:qp")


def test_dummy_address_and_current_encoding():
    """reference guiutiltests.cpp dummyAddressTest / toCurrentEncodingTest"""
    for cash in (False, True):
        d = native.dummy_address(cash)
        assert d and not native.is_valid_destination(d)
    assert native.dummy_address(True).startswith("bitcoincashplus:")
    cash_addr = "bitcoincashplus:qqqprqq976hvnqkeajpc33u5rt92xw5vm5ylgfku0f"
    b58 = "CGUFXy9eQgs3eunVAEqFdS9tnkEcgLw9VD"
    assert native.to_current_encoding("garbage", True) == "garbage"
    assert native.to_current_encoding(cash_addr, True) == cash_addr
    assert native.to_current_encoding(b58, True) == cash_addr
    assert native.to_current_encoding(cash_addr, False) == b58
    assert native.to_current_encoding(b58, False) == b58
