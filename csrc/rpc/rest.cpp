// REST interface (-rest). Parity: reference src/rest.cpp: /rest/tx/<txid>.<fmt>,
// /rest/block/<hash>.<fmt>, /rest/block/notxdetails/<hash>.<fmt>, /rest/chaininfo.json,
// /rest/mempool/info.json, /rest/mempool/contents.json, /rest/headers/<count>/<hash>.<fmt>,
// /rest/getutxos[/checkmempool]/<txid>-<n>/....<fmt> (formats bin|hex|json).
#include "node/node.h"
#include "node/txmempool.h"
#include "rpc/core_io.h"
#include "rpc/httpserver.h"
#include "rpc/server.h"
#include "util/strencodings.h"

namespace bcp {

UniValue blockToJSON(const CBlock& block, const CBlockIndex* blockindex, bool txDetails);
UniValue blockheaderToJSON(const CBlockIndex* blockindex);
UniValue mempoolInfoToJSON();
UniValue mempoolToJSON(bool fVerbose);

enum RetFormat { RF_UNDEF, RF_BINARY, RF_HEX, RF_JSON };

static RetFormat ParseDataFormat(std::string& param, const std::string& strReq) {
    const size_t pos = strReq.rfind('.');
    if (pos == std::string::npos) {
        param = strReq;
        return RF_UNDEF;
    }
    param = strReq.substr(0, pos);
    const std::string suff = strReq.substr(pos + 1);
    if (suff == "bin") return RF_BINARY;
    if (suff == "hex") return RF_HEX;
    if (suff == "json") return RF_JSON;
    return RF_UNDEF;
}

static bool RESTERR(HTTPReply& rep, int status, const std::string& message) {
    rep.status = status;
    rep.contentType = "text/plain";
    rep.body = message + "\r\n";
    return false;
}

static bool Reply(HTTPReply& rep, RetFormat rf, const std::vector<unsigned char>& bin, const UniValue& json) {
    switch (rf) {
    case RF_BINARY:
        rep.contentType = "application/octet-stream";
        rep.body.assign(bin.begin(), bin.end());
        return true;
    case RF_HEX:
        rep.contentType = "text/plain";
        rep.body = HexStr(bin) + "\n";
        return true;
    case RF_JSON:
        rep.contentType = "application/json";
        rep.body = json.write() + "\n";
        return true;
    default: return RESTERR(rep, 404, "output format not found (available: bin, hex, json)");
    }
}

static bool rest_block(const HTTPRequest& req, HTTPReply& rep, const std::string& strURIPart, bool showTxDetails) {
    NodeContext* n = GetNode();
    std::string hashStr;
    const RetFormat rf = ParseDataFormat(hashStr, strURIPart);
    if (hashStr.size() != 64 || !IsHex(hashStr)) return RESTERR(rep, 400, "Invalid hash: " + hashStr);
    const uint256 hash = uint256S(hashStr);
    Chainstate& cs = *n->chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    CBlockIndex* pindex = cs.LookupBlockIndex(hash);
    if (!pindex) return RESTERR(rep, 404, hashStr + " not found");
    if (cs.HavePruned() && !(pindex->nStatus & BLOCK_HAVE_DATA) && pindex->nTx > 0)
        return RESTERR(rep, 404, hashStr + " not available (pruned data)");
    CBlock block;
    if (!cs.ReadBlock(block, pindex)) return RESTERR(rep, 404, hashStr + " not found");
    const bool legacy = pindex->nHeight < cs.Params().GetConsensus().BCPHeight;
    return Reply(rep, rf, SerializeToBytes(block, SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0)),
                 rf == RF_JSON ? blockToJSON(block, pindex, showTxDetails) : UniValue());
}

static bool rest_tx(const HTTPRequest& req, HTTPReply& rep, const std::string& strURIPart) {
    NodeContext* n = GetNode();
    std::string hashStr;
    const RetFormat rf = ParseDataFormat(hashStr, strURIPart);
    if (hashStr.size() != 64 || !IsHex(hashStr)) return RESTERR(rep, 400, "Invalid hash: " + hashStr);
    CTransactionRef tx;
    uint256 hashBlock;
    if (!n->chainstate->GetTransaction(uint256S(hashStr), tx, hashBlock, true)) return RESTERR(rep, 404, hashStr + " not found");
    UniValue obj(UniValue::VOBJ);
    if (rf == RF_JSON) TxToUniv(*tx, hashBlock, obj, n->chainstate->Params(), false);
    return Reply(rep, rf, SerializeToBytes(*tx), obj);
}

static bool rest_headers(const HTTPRequest& req, HTTPReply& rep, const std::string& strURIPart) {
    NodeContext* n = GetNode();
    std::string param;
    const RetFormat rf = ParseDataFormat(param, strURIPart);
    std::vector<std::string> path = SplitString(param, '/');
    if (path.size() != 2) return RESTERR(rep, 400, "No header count specified. Use /rest/headers/<count>/<hash>.<ext>.");
    const long count = strtol(path[0].c_str(), nullptr, 10);
    if (count < 1 || count > 2000) return RESTERR(rep, 400, "Header count out of range: " + path[0]);
    if (path[1].size() != 64 || !IsHex(path[1])) return RESTERR(rep, 400, "Invalid hash: " + path[1]);
    Chainstate& cs = *n->chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    std::vector<const CBlockIndex*> headers;
    const CBlockIndex* pindex = cs.LookupBlockIndex(uint256S(path[1]));
    while (pindex != nullptr && cs.ActiveChain().Contains(pindex)) {
        headers.push_back(pindex);
        if ((long)headers.size() == count) break;
        pindex = cs.ActiveChain().Next(pindex);
    }
    std::vector<unsigned char> bin;
    UniValue arr(UniValue::VARR);
    for (const CBlockIndex* p : headers) {
        const bool legacy = p->nHeight < cs.Params().GetConsensus().BCPHeight;
        std::vector<unsigned char> h = SerializeToBytes(p->GetBlockHeader(), SER_NETWORK,
                                                        PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0));
        bin.insert(bin.end(), h.begin(), h.end());
        if (rf == RF_JSON) arr.push_back(blockheaderToJSON(p));
    }
    return Reply(rep, rf, bin, arr);
}

static bool rest_getutxos(const HTTPRequest& req, HTTPReply& rep, const std::string& strURIPart) {
    NodeContext* n = GetNode();
    std::string param;
    const RetFormat rf = ParseDataFormat(param, strURIPart);
    std::vector<std::string> uriParts;
    if (!param.empty()) uriParts = SplitString(param.substr(1), '/');
    bool fCheckMemPool = false;
    std::vector<COutPoint> vOutPoints;
    if (!uriParts.empty() && uriParts[0] == "checkmempool") {
        fCheckMemPool = true;
        uriParts.erase(uriParts.begin());
    }
    for (const std::string& part : uriParts) {
        const size_t dash = part.find('-');
        if (dash == std::string::npos) return RESTERR(rep, 400, "Parse error");
        const std::string txid = part.substr(0, dash);
        if (txid.size() != 64 || !IsHex(txid)) return RESTERR(rep, 400, "Parse error");
        vOutPoints.push_back(COutPoint(uint256S(txid), (uint32_t)atoi(part.substr(dash + 1).c_str())));
    }
    if (vOutPoints.empty()) return RESTERR(rep, 400, "Error: empty request");
    if (vOutPoints.size() > 15) return RESTERR(rep, 400, "Error: max outpoints exceeded (max: 15, tried: " + std::to_string(vOutPoints.size()) + ")");
    Chainstate& cs = *n->chainstate;
    std::vector<unsigned char> bitmap((vOutPoints.size() + 7) / 8);
    std::vector<Coin> outs;
    std::string bitmapStringRepresentation;
    int chainHeight; // the tip the lookups were made against (same cs_main scope)
    uint256 tipHash;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        chainHeight = cs.Height();
        tipHash = cs.Tip()->GetBlockHash();
        std::lock_guard<CCriticalSection> lm(n->mempool->cs);
        CCoinsViewMemPool viewMempool(&cs.CoinsTip(), *n->mempool);
        CCoinsView& view = fCheckMemPool ? static_cast<CCoinsView&>(viewMempool) : static_cast<CCoinsView&>(cs.CoinsTip());
        for (size_t i = 0; i < vOutPoints.size(); i++) {
            Coin coin;
            const bool hit = view.GetCoin(vOutPoints[i], coin) && !coin.IsSpent() &&
                             !(fCheckMemPool && n->mempool->isSpent(vOutPoints[i]));
            if (hit) {
                outs.push_back(coin);
                bitmap[i / 8] |= 1 << (i % 8);
            }
            bitmapStringRepresentation += hit ? "1" : "0";
        }
    }
    std::vector<unsigned char> bin;
    {
        VectorWriter w(bin);
        w << (int32_t)chainHeight << tipHash << bitmap;
        WriteCompactSize(w, outs.size());
        for (const Coin& c : outs) w << (uint32_t)c.nHeight << c.out;
    }
    UniValue objGetUTXOResponse(UniValue::VOBJ);
    objGetUTXOResponse.pushKV("chainHeight", chainHeight);
    objGetUTXOResponse.pushKV("chaintipHash", tipHash.GetHex());
    objGetUTXOResponse.pushKV("bitmap", bitmapStringRepresentation);
    UniValue utxos(UniValue::VARR);
    for (const Coin& c : outs) {
        UniValue utxo(UniValue::VOBJ);
        utxo.pushKV("height", (int32_t)c.nHeight);
        utxo.pushKV("value", ValueFromAmount(c.out.nValue));
        UniValue o(UniValue::VOBJ);
        ScriptPubKeyToUniv(c.out.scriptPubKey, o, true, cs.Params());
        utxo.pushKV("scriptPubKey", o);
        utxos.push_back(utxo);
    }
    objGetUTXOResponse.pushKV("utxos", utxos);
    return Reply(rep, rf, bin, objGetUTXOResponse);
}

void StartREST(HTTPServer& server) {
    server.RegisterHandler("/rest/", false, [](const HTTPRequest& req, HTTPReply& rep) -> bool {
        if (!GetNode() || !GetNode()->chainstate) return RESTERR(rep, 503, "Service temporarily unavailable");
        std::string status;
        if (RPCIsInWarmup(&status)) return RESTERR(rep, 503, "Service temporarily unavailable: " + status);
        const std::string& uri = req.uri;
        auto starts = [&](const char* p) { return uri.compare(0, strlen(p), p) == 0; };
        if (starts("/rest/block/notxdetails/")) return rest_block(req, rep, uri.substr(strlen("/rest/block/notxdetails/")), false);
        if (starts("/rest/block/")) return rest_block(req, rep, uri.substr(strlen("/rest/block/")), true);
        if (starts("/rest/tx/")) return rest_tx(req, rep, uri.substr(strlen("/rest/tx/")));
        if (starts("/rest/headers/")) return rest_headers(req, rep, uri.substr(strlen("/rest/headers/")));
        if (starts("/rest/getutxos")) return rest_getutxos(req, rep, uri.substr(strlen("/rest/getutxos")));
        if (starts("/rest/chaininfo")) {
            std::string p;
            if (ParseDataFormat(p, uri) != RF_JSON) return RESTERR(rep, 404, "output format not found (available: json)");
            JSONRPCRequest jr;
            jr.strMethod = "getblockchaininfo";
            jr.params = UniValue(UniValue::VARR);
            UniValue r = tableRPC.execute(jr);
            return Reply(rep, RF_JSON, {}, r);
        }
        if (starts("/rest/mempool/info")) {
            std::string p;
            if (ParseDataFormat(p, uri) != RF_JSON) return RESTERR(rep, 404, "output format not found (available: json)");
            return Reply(rep, RF_JSON, {}, mempoolInfoToJSON());
        }
        if (starts("/rest/mempool/contents")) {
            std::string p;
            if (ParseDataFormat(p, uri) != RF_JSON) return RESTERR(rep, 404, "output format not found (available: json)");
            return Reply(rep, RF_JSON, {}, mempoolToJSON(true));
        }
        return RESTERR(rep, 404, "not found");
    });
}

} // namespace bcp
