// BIP21 payment URIs ("<scheme>:<address>?amount=..&label=..&message=..", BIP72 r=).
//
// Parity: reference src/qt/guiutil.cpp parseBitcoinURI (:185-257), formatBitcoinURI (:259-289),
// bitcoinURIScheme (:168-177) and BitcoinUnits::parse for the BCP unit, tested by
// src/qt/test/uritests.cpp. The reference parses through QUrl/QUrlQuery inside the Qt GUI;
// here the same rules are plain C++ used by the browser GUI (RPC parsebitcoinuri /
// formatbitcoinuri) and the tests.
#pragma once

#include "consensus/params.h"
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

// Address entry helpers of the send form (reference src/qt/bitcoinaddressvalidator.cpp
// BitcoinAddressEntryValidator::validate, src/qt/guiutil.cpp DummyAddress and
// ToCurrentEncoding, tested by bitcoinaddressvalidatortests.cpp and guiutiltests.cpp).
enum class AddressInputState { Invalid, Intermediate, Acceptable };
// Drops whitespace and zero-width spaces from `input` (UTF-8), then accepts only [0-9A-Za-z:].
AddressInputState ValidateAddressInput(std::string& input);
// A plausible-looking placeholder address that is not valid, in the selected encoding.
std::string DummyAddress(const CChainParams& params, bool useCashAddr);
// A valid address re-encoded in the selected encoding; anything else unchanged.
std::string ToCurrentEncoding(const std::string& addr, const CChainParams& params, bool useCashAddr);

} // namespace bcp
