// BIP21 payment URIs ("<scheme>:<address>?amount=..&label=..&message=..", BIP72 r=).
//
// Parity: reference src/qt/guiutil.cpp parseBitcoinURI (:185-257), formatBitcoinURI (:259-289),
// bitcoinURIScheme (:168-177) and BitcoinUnits::parse for the BCP unit, tested by
// src/qt/test/uritests.cpp. The reference parses through QUrl/QUrlQuery inside the Qt GUI;
// here the same rules are plain C++ used by the browser GUI (RPC parsebitcoinuri /
// formatbitcoinuri) and the tests.
#pragma once

#include "primitives/amount.h"

#include <string>

namespace bcp {

struct SendCoinsRecipient {
    std::string address;
    std::string label;
    std::string message;
    std::string paymentRequestUrl; // BIP72 r= (fetched by the payment request flow)
    Amount amount = 0;
};

// Decimal coin amount with at most 8 fractional digits and no separators ("1.001" ->
// 100100000); false on anything else, including values too large for 63 bits.
bool ParseCoinAmount(const std::string& text, Amount* out);

// The scheme of URIs for this chain: the CashAddr prefix, or "bitcoincashplus" without CashAddr.
std::string BitcoinURIScheme(bool useCashAddr);

// Parses `uri` for `scheme`; "scheme://addr" is accepted as "scheme:addr". Unknown req-*
// parameters, a malformed amount or a wrong scheme make it fail. A CashAddr address keeps its
// prefix, a Base58 address does not.
bool ParseBitcoinURI(const std::string& scheme, const std::string& uri, SendCoinsRecipient* out);

std::string FormatBitcoinURI(const SendCoinsRecipient& info, bool useCashAddr);

} // namespace bcp
