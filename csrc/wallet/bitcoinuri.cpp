// BIP21 payment URIs (see bitcoinuri.h for parity).
#include "wallet/bitcoinuri.h"

#include "consensus/params.h"
#include "keys/key.h"

#include <cctype>
#include <vector>

namespace bcp {

namespace {

std::string PercentDecode(const std::string& s) {
    std::string out;
    for (size_t i = 0; i < s.size(); i++) {
        if (s[i] == '%' && i + 2 < s.size() && std::isxdigit((unsigned char)s[i + 1]) &&
            std::isxdigit((unsigned char)s[i + 2])) {
            out += (char)std::stoi(s.substr(i + 1, 2), nullptr, 16);
            i += 2;
        } else {
            out += s[i];
        }
    }
    return out;
}

std::string PercentEncode(const std::string& s) {
    static const char* hex = "0123456789ABCDEF";
    std::string out;
    for (unsigned char c : s) {
        if (std::isalnum(c) || c == '-' || c == '.' || c == '_' || c == '~') {
            out += (char)c;
        } else {
            out += '%';
            out += hex[c >> 4];
            out += hex[c & 15];
        }
    }
    return out;
}

std::string Lower(std::string s) {
    for (char& c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

std::string FormatCoins(Amount a) {
    const bool neg = a < 0;
    const uint64_t v = neg ? (uint64_t)(-(a + 1)) + 1 : (uint64_t)a;
    std::string frac = std::to_string(v % COIN);
    frac.insert(0, 8 - frac.size(), '0');
    while (!frac.empty() && frac.back() == '0') frac.pop_back();
    std::string r = (neg ? "-" : "") + std::to_string(v / COIN);
    if (!frac.empty()) r += "." + frac;
    return r;
}

} // namespace

bool ParseCoinAmount(const std::string& text, Amount* out) {
    std::string t;
    for (char c : text)
        if (c != ' ') t += c; // spaces (digit grouping) are ignored, as in BitcoinUnits::parse
    if (t.empty()) return false;
    const size_t dot = t.find('.');
    if (dot != std::string::npos && t.find('.', dot + 1) != std::string::npos) return false;
    const std::string whole = t.substr(0, dot), dec = dot == std::string::npos ? "" : t.substr(dot + 1);
    if (dec.size() > 8) return false;
    const std::string digits = whole + dec + std::string(8 - dec.size(), '0');
    if (digits.size() > 18) return false; // beyond 63 bits
    for (char c : digits)
        if (!std::isdigit((unsigned char)c)) return false;
    if (out) *out = (Amount)std::stoll(digits);
    return true;
}

std::string BitcoinURIScheme(bool useCashAddr) { return useCashAddr ? Params().CashAddrPrefix() : "bitcoincashplus"; }

bool ParseBitcoinURI(const std::string& scheme, const std::string& uriIn, SendCoinsRecipient* out) {
    std::string uri = uriIn;
    // "scheme://addr" would make a URL parser lower-case the address as a host name
    if (Lower(uri.substr(0, scheme.size() + 3)) == Lower(scheme) + "://") uri.replace(0, scheme.size() + 3, scheme + ":");
    const size_t colon = uri.find(':');
    if (colon == std::string::npos || colon == 0) return false;
    const std::string uriScheme = Lower(uri.substr(0, colon));
    for (char c : uriScheme)
        if (!(std::isalnum((unsigned char)c) || c == '+' || c == '-' || c == '.')) return false;
    if (uriScheme != scheme) return false;
    const size_t q = uri.find('?', colon + 1);
    const size_t frag = uri.find('#', colon + 1);
    std::string path = PercentDecode(uri.substr(colon + 1, (q == std::string::npos ? frag : q) - colon - 1));
    std::string query = q == std::string::npos ? "" : uri.substr(q + 1, frag == std::string::npos ? std::string::npos : frag - q - 1);

    SendCoinsRecipient rv;
    const std::string prefixed = uriScheme + ":" + path;
    rv.address = cashaddr::Decode(prefixed, "").first.empty() ? path : prefixed;
    if (!rv.address.empty() && rv.address.back() == '/') rv.address.pop_back();

    size_t start = 0;
    while (start <= query.size() && !query.empty()) {
        const size_t amp = query.find('&', start);
        const std::string item = query.substr(start, amp == std::string::npos ? std::string::npos : amp - start);
        start = amp == std::string::npos ? query.size() + 1 : amp + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        std::string key = PercentDecode(item.substr(0, eq));
        const std::string value = eq == std::string::npos ? "" : PercentDecode(item.substr(eq + 1));
        bool required = false;
        if (key.compare(0, 4, "req-") == 0) {
            key.erase(0, 4);
            required = true;
        }
        if (key == "label") {
            rv.label = value;
        } else if (key == "message") {
            rv.message = value;
        } else if (key == "amount") {
            if (!value.empty() && !ParseCoinAmount(value, &rv.amount)) return false;
        } else if (key == "r") {
            rv.paymentRequestUrl = value;
        } else if (required) {
            return false; // a required parameter this wallet does not understand
        }
    }
    if (out) *out = rv;
    return true;
}

std::string FormatBitcoinURI(const SendCoinsRecipient& info, bool useCashAddr) {
    std::string ret = useCashAddr ? info.address : BitcoinURIScheme(false) + ":" + info.address;
    const char* sep = "?";
    if (info.amount != 0) {
        ret += std::string(sep) + "amount=" + FormatCoins(info.amount);
        sep = "&";
    }
    if (!info.label.empty()) {
        ret += std::string(sep) + "label=" + PercentEncode(info.label);
        sep = "&";
    }
    if (!info.message.empty()) ret += std::string(sep) + "message=" + PercentEncode(info.message);
    return ret;
}

AddressInputState ValidateAddressInput(std::string& input) {
    if (input.empty()) return AddressInputState::Intermediate;
    std::string kept;
    for (size_t i = 0; i < input.size();) {
        const unsigned char c = (unsigned char)input[i];
        // U+200B ZERO WIDTH SPACE (e2 80 8b), U+FEFF ZERO WIDTH NO-BREAK SPACE (ef bb bf)
        if (input.compare(i, 3, "\xe2\x80\x8b") == 0 || input.compare(i, 3, "\xef\xbb\xbf") == 0) {
            i += 3;
            continue;
        }
        if (std::isspace(c)) {
            i++;
            continue;
        }
        kept += (char)c;
        i++;
    }
    input = kept;
    for (unsigned char c : input)
        if (!(std::isalnum(c) && c < 0x80) && c != ':') return AddressInputState::Invalid;
    return AddressInputState::Acceptable;
}

std::string DummyAddress(const CChainParams& params, bool useCashAddr) {
    static const std::vector<unsigned char> data = {0x3a, 0x91, 0x07, 0xc4, 0x5e, 0x2b, 0xd8, 0x60, 0x19, 0xf3,
                                                    0x44, 0xa7, 0x0c, 0x82, 0x6d, 0xe5, 0x31, 0x9b, 0x58, 0x0f};
    const CTxDestination d{CKeyID(uint160(data))};
    std::string addr = useCashAddr ? EncodeCashAddr(d, params) : EncodeLegacyAddr(d, params);
    // change the last character until the checksum no longer matches
    static const std::string alphabet = "qpzry9x8gf2tvdw0s3jn54khce6mua7l";
    const char orig = addr.back();
    for (char c : alphabet) {
        if (c == orig) continue;
        addr.back() = c;
        if (!IsValidDestinationString(addr, params)) break;
    }
    return addr;
}

std::string ToCurrentEncoding(const std::string& addr, const CChainParams& params, bool useCashAddr) {
    const CTxDestination d = DecodeDestination(addr, params);
    if (!d.IsValid()) return addr;
    return useCashAddr ? EncodeCashAddr(d, params) : EncodeLegacyAddr(d, params);
}

} // namespace bcp
