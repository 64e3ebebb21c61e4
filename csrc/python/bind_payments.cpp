// Python bindings: BIP70 payment protocol (wallet/paymentrequest.h) for tests.
#include "python/bind.h"
#include "keys/key.h"
#include "wallet/bitcoinuri.h"
#include "wallet/paymentrequest.h"

namespace bcp {
namespace py {

using namespace payments;

void bind_payments(pyb::module_& m) {
    m.attr("BIP70_MAX_PAYMENTREQUEST_SIZE") = BIP70_MAX_PAYMENTREQUEST_SIZE;
    // Parse a serialized PaymentRequest and run the wallet's checks on it: merchant
    // authentication against `roots` (DER) at time `now`, network, expiry, amounts.
    m.def(
        "payment_request_info",
        [](const pyb::bytes& data, const std::vector<pyb::bytes>& roots, const std::string& network, int64_t now,
           bool allowSelfSigned) {
            const std::string raw = data;
            pyb::dict r;
            r["size_ok"] = VerifySize((int64_t)raw.size());
            PaymentRequestPlus pr;
            r["initialized"] = pr.parse(raw);
            if (!pr.IsInitialized()) return r;
            CertStore cs;
            for (const auto& b : roots) cs.roots_der.push_back(std::string(b));
            cs.now = now;
            cs.allow_self_signed_root = allowSelfSigned;
            std::string merchant, err;
            pr.getMerchant(cs, merchant, &err);
            const PaymentDetails& d = pr.getDetails();
            r["merchant"] = merchant;
            r["merchant_error"] = err;
            r["pki_type"] = pr.getRequest().pki_type;
            r["version"] = pr.getRequest().payment_details_version;
            r["network"] = d.network;
            r["network_ok"] = VerifyNetwork(d, network);
            r["expired"] = VerifyExpired(d, now);
            r["time"] = d.time;
            r["expires"] = d.has_expires ? pyb::cast(d.expires) : pyb::none();
            r["memo"] = d.memo;
            r["payment_url"] = d.payment_url;
            r["merchant_data"] = pyb::bytes(d.merchant_data);
            pyb::list outs;
            for (const auto& [script, amount] : pr.getPayTo())
                outs.append(pyb::make_tuple(to_bytes(script.data(), script.size()), amount, VerifyAmount(amount)));
            r["outputs"] = outs;
            r["reserialized"] = pyb::bytes(pr.SerializeToString());
            return r;
        },
        pyb::arg("data"), pyb::arg("roots") = std::vector<pyb::bytes>{}, pyb::arg("network") = "main",
        pyb::arg("now") = 0, pyb::arg("allow_self_signed") = false);
    // Build a PaymentRequest (signature left out; see payment_request_signing_data).
    m.def(
        "payment_request_build",
        [](const std::vector<std::pair<uint64_t, pyb::bytes>>& outputs, uint64_t time, pyb::object expires,
           const std::string& network, const std::string& memo, const std::string& paymentUrl,
           const pyb::bytes& merchantData, const std::string& pkiType, const std::vector<pyb::bytes>& chain,
           uint32_t version) {
            PaymentDetails d;
            d.has_network = true;
            d.network = network;
            for (const auto& [amount, script] : outputs) {
                Output o;
                o.has_amount = o.has_script = true;
                o.amount = amount;
                o.script = std::string(script);
                d.outputs.push_back(o);
            }
            d.has_time = true;
            d.time = time;
            if (!expires.is_none()) {
                d.has_expires = true;
                d.expires = expires.cast<uint64_t>();
            }
            d.has_memo = !memo.empty();
            d.memo = memo;
            d.has_payment_url = !paymentUrl.empty();
            d.payment_url = paymentUrl;
            d.merchant_data = std::string(merchantData);
            d.has_merchant_data = !d.merchant_data.empty();
            PaymentRequest q;
            q.has_version = true;
            q.payment_details_version = version;
            q.has_pki_type = true;
            q.pki_type = pkiType;
            if (!chain.empty()) {
                std::vector<std::string> c;
                for (const auto& b : chain) c.push_back(std::string(b));
                q.has_pki_data = true;
                q.pki_data = SerializeX509Certificates(c);
            }
            q.has_details = true;
            q.serialized_payment_details = SerializePaymentDetails(d);
            return pyb::bytes(SerializePaymentRequest(q));
        },
        pyb::arg("outputs"), pyb::arg("time"), pyb::arg("expires") = pyb::none(), pyb::arg("network") = "main",
        pyb::arg("memo") = "", pyb::arg("payment_url") = "", pyb::arg("merchant_data") = pyb::bytes(""),
        pyb::arg("pki_type") = "none", pyb::arg("chain") = std::vector<pyb::bytes>{}, pyb::arg("version") = 1);
    // The bytes a merchant signs: the request with an empty signature field.
    m.def("payment_request_signing_data", [](const pyb::bytes& data) {
        PaymentRequest q;
        if (!ParsePaymentRequest(std::string(data), q)) throw std::invalid_argument("bad payment request");
        q.signature.clear();
        q.has_signature = true;
        return pyb::bytes(SerializePaymentRequest(q));
    });
    m.def("payment_request_set_signature", [](const pyb::bytes& data, const pyb::bytes& sig) {
        PaymentRequest q;
        if (!ParsePaymentRequest(std::string(data), q)) throw std::invalid_argument("bad payment request");
        q.signature = std::string(sig);
        q.has_signature = true;
        return pyb::bytes(SerializePaymentRequest(q));
    });
    // BIP21 URIs: (ok, address, amount, label, message, r)
    m.def("parse_bitcoin_uri", [](const std::string& scheme, const std::string& uri) {
        SendCoinsRecipient r;
        const bool ok = ParseBitcoinURI(scheme, uri, &r);
        return pyb::make_tuple(ok, r.address, r.amount, r.label, r.message, r.paymentRequestUrl);
    });
    m.def(
        "format_bitcoin_uri",
        [](const std::string& address, Amount amount, const std::string& label, const std::string& message,
           bool useCashAddr) {
            SendCoinsRecipient r;
            r.address = address;
            r.amount = amount;
            r.label = label;
            r.message = message;
            return FormatBitcoinURI(r, useCashAddr);
        },
        pyb::arg("address"), pyb::arg("amount") = 0, pyb::arg("label") = "", pyb::arg("message") = "",
        pyb::arg("use_cashaddr") = true);
    m.def("validate_address_input", [](std::string input) {
        const AddressInputState st = ValidateAddressInput(input);
        return pyb::make_tuple(st == AddressInputState::Invalid ? "invalid"
                               : st == AddressInputState::Intermediate ? "intermediate" : "acceptable", input);
    });
    m.def(
        "dummy_address", [](bool cash, const std::string& chain) { return DummyAddress(Params(chain), cash); },
        pyb::arg("use_cashaddr"), pyb::arg("chain") = "main");
    m.def(
        "to_current_encoding",
        [](const std::string& a, bool cash, const std::string& chain) { return ToCurrentEncoding(a, Params(chain), cash); },
        pyb::arg("address"), pyb::arg("use_cashaddr"), pyb::arg("chain") = "main");
    m.def("is_valid_destination", [](const std::string& a, const std::string& chain) {
        return IsValidDestinationString(a, Params(chain));
    }, pyb::arg("address"), pyb::arg("chain") = "main");
    m.def("parse_coin_amount", [](const std::string& t) -> pyb::object {
        Amount a;
        if (!ParseCoinAmount(t, &a)) return pyb::none();
        return pyb::cast(a);
    });
    // Payment / PaymentACK round trips (what sendpaymentrequest hands back for payment_url).
    m.def("payment_decode", [](const pyb::bytes& data) {
        Payment p;
        if (!ParsePayment(std::string(data), p)) throw std::invalid_argument("bad payment");
        pyb::dict r;
        r["merchant_data"] = pyb::bytes(p.merchant_data);
        pyb::list txs, refunds;
        for (const auto& t : p.transactions) txs.append(pyb::bytes(t));
        for (const auto& o : p.refund_to) refunds.append(pyb::make_tuple(o.amount, pyb::bytes(o.script)));
        r["transactions"] = txs;
        r["refund_to"] = refunds;
        r["memo"] = p.memo;
        return r;
    });
    m.def("payment_ack_roundtrip", [](const pyb::bytes& payment, const std::string& memo) {
        PaymentACK a;
        if (!ParsePayment(std::string(payment), a.payment)) throw std::invalid_argument("bad payment");
        a.has_memo = !memo.empty();
        a.memo = memo;
        const std::string s = SerializePaymentACK(a);
        PaymentACK b;
        if (!ParsePaymentACK(s, b)) throw std::runtime_error("PaymentACK did not parse back");
        return pyb::make_tuple(pyb::bytes(s), pyb::bytes(SerializePayment(b.payment)), b.memo);
    });
}

} // namespace py
} // namespace bcp
