// Raw transaction RPCs. Parity: reference src/rpc/rawtransaction.cpp (command table
// :1167): getrawtransaction, createrawtransaction, decoderawtransaction, decodescript,
// sendrawtransaction, signrawtransaction (FORKID required :981-1013, prevtxs amount
// mandatory :938-948), gettxoutproof, verifytxoutproof.
#include "consensus/merkleblock.h"
#include "keys/key.h"
#include "node/node.h"
#include "node/policy.h"
#include "node/signals.h"
#include "node/txmempool.h"
#include "rpc/core_io.h"
#include "rpc/server.h"
#include "script/sign.h"
#include "script/standard.h"
#include "util/strencodings.h"

namespace bcp {

static NodeContext& Node() {
    NodeContext* n = GetNode();
    if (!n || !n->chainstate) ThrowRPC(RPC_INTERNAL_ERROR, "node not initialised");
    return *n;
}

// Relay hook set by the P2P layer (announce a tx to peers).
std::function<void(const uint256&)> g_relayTransaction;

static UniValue getrawtransaction(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "getrawtransaction \"txid\" ( verbose )");
    NodeContext& n = Node();
    const uint256 hash = ParseHashV(req.params[0], "parameter 1");
    bool fVerbose = false;
    if (req.params.size() > 1 && !req.params[1].isNull()) {
        if (req.params[1].isNum()) fVerbose = req.params[1].get_int() != 0;
        else if (req.params[1].isBool()) fVerbose = req.params[1].isTrue();
        else ThrowRPC(RPC_TYPE_ERROR, "Invalid type provided. Verbose parameter must be a boolean.");
    }
    CTransactionRef tx;
    uint256 hashBlock;
    if (!n.chainstate->GetTransaction(hash, tx, hashBlock, true))
        ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY,
                 std::string(n.chainstate->TxIndexEnabled() ? "No such mempool or blockchain transaction"
                                                             : "No such mempool transaction. Use -txindex to enable blockchain transaction queries") +
                     ". Use gettransaction for wallet transactions.");
    const std::string strHex = EncodeHexTx(*tx);
    if (!fVerbose) return strHex;
    UniValue result(UniValue::VOBJ);
    result.pushKV("hex", strHex);
    TxToUniv(*tx, hashBlock, result, n.chainstate->Params());
    if (!hashBlock.IsNull()) {
        std::lock_guard<CCriticalSection> l(n.chainstate->cs());
        CBlockIndex* pindex = n.chainstate->LookupBlockIndex(hashBlock);
        if (pindex) {
            if (n.chainstate->ActiveChain().Contains(pindex)) {
                result.pushKV("confirmations", 1 + n.chainstate->Height() - pindex->nHeight);
                result.pushKV("time", pindex->GetBlockTime());
                result.pushKV("blocktime", pindex->GetBlockTime());
            } else {
                result.pushKV("confirmations", 0);
            }
        }
    }
    return result;
}

static UniValue createrawtransaction(const JSONRPCRequest& req) {
    if (req.params.size() < 2 || req.params.size() > 3)
        ThrowRPC(RPC_INVALID_PARAMS, "createrawtransaction [{\"txid\":\"id\",\"vout\":n},...] {\"address\":amount,\"data\":\"hex\",...} ( locktime )");
    RPCTypeCheck(req.params, {UniValue::VARR, UniValue::VOBJ, UniValue::VNUM}, true);
    if (req.params[0].isNull() || req.params[1].isNull())
        ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, arguments 1 and 2 must be non-null");
    const CChainParams& params = Node().chainstate->Params();
    const UniValue& inputs = req.params[0].get_array();
    const UniValue& sendTo = req.params[1].get_obj();
    CMutableTransaction rawTx;
    if (req.params.size() > 2 && !req.params[2].isNull()) {
        const int64_t nLockTime = req.params[2].get_int64();
        if (nLockTime < 0 || nLockTime > 0xFFFFFFFFLL) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, locktime out of range");
        rawTx.nLockTime = (uint32_t)nLockTime;
    }
    for (size_t idx = 0; idx < inputs.size(); idx++) {
        const UniValue& o = inputs[idx].get_obj();
        const uint256 txid = ParseHashO(o, "txid");
        const UniValue& vout_v = o["vout"];
        if (!vout_v.isNum()) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, missing vout key");
        const int nOutput = vout_v.get_int();
        if (nOutput < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, vout must be positive");
        uint32_t nSequence = rawTx.nLockTime ? (CTxIn::SEQUENCE_FINAL - 1) : CTxIn::SEQUENCE_FINAL;
        const UniValue& sequenceObj = o["sequence"];
        if (sequenceObj.isNum()) {
            const int64_t seqNr64 = sequenceObj.get_int64();
            if (seqNr64 < 0 || seqNr64 > CTxIn::SEQUENCE_FINAL)
                ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, sequence number is out of range");
            nSequence = (uint32_t)seqNr64;
        }
        rawTx.vin.push_back(CTxIn(COutPoint(txid, (uint32_t)nOutput), CScript(), nSequence));
    }
    std::set<CTxDestination> destinations;
    for (const std::string& name_ : sendTo.getKeys()) {
        if (name_ == "data") {
            std::vector<unsigned char> data = ParseHexV(sendTo[name_], "Data");
            CScript s;
            s << OP_RETURN << data;
            rawTx.vout.push_back(CTxOut(0, s));
        } else {
            CTxDestination dest = DecodeDestination(name_, params);
            if (!dest.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address: " + name_);
            if (!destinations.insert(dest).second) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated address: " + name_);
            rawTx.vout.push_back(CTxOut(AmountFromValue(sendTo[name_]), GetScriptForDestination(dest)));
        }
    }
    return EncodeHexTx(CTransaction(rawTx));
}

static UniValue decoderawtransaction(const JSONRPCRequest& req) {
    RPCTypeCheck(req.params, {UniValue::VSTR});
    CMutableTransaction mtx;
    if (!DecodeHexTx(mtx, req.params[0].get_str())) ThrowRPC(RPC_DESERIALIZATION_ERROR, "TX decode failed");
    UniValue result(UniValue::VOBJ);
    TxToUniv(CTransaction(std::move(mtx)), uint256(), result, Node().chainstate->Params());
    return result;
}

static UniValue decodescript(const JSONRPCRequest& req) {
    RPCTypeCheck(req.params, {UniValue::VSTR});
    const CChainParams& params = Node().chainstate->Params();
    UniValue r(UniValue::VOBJ);
    CScript script;
    if (req.params[0].get_str().size() > 0) {
        std::vector<unsigned char> scriptData(ParseHexV(req.params[0], "argument"));
        script = CScript(scriptData.begin(), scriptData.end());
    }
    ScriptPubKeyToUniv(script, r, false, params);
    UniValue type = r["type"];
    if (type.isStr() && type.get_str() != "scripthash")
        r.pushKV("p2sh", EncodeDestination(CTxDestination(CScriptID(script)), params));
    return r;
}

static void TxInErrorToJSON(const CTxIn& txin, UniValue& vErrorsRet, const std::string& strMessage) {
    UniValue entry(UniValue::VOBJ);
    entry.pushKV("txid", txin.prevout.hash.ToString());
    entry.pushKV("vout", (uint64_t)txin.prevout.n);
    entry.pushKV("scriptSig", HexStr(txin.scriptSig.begin(), txin.scriptSig.end()));
    entry.pushKV("sequence", (uint64_t)txin.nSequence);
    entry.pushKV("error", strMessage);
    vErrorsRet.push_back(entry);
}

static UniValue signrawtransaction(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 4)
        ThrowRPC(RPC_INVALID_PARAMS, "signrawtransaction \"hexstring\" ( [{\"txid\":\"id\",\"vout\":n,\"scriptPubKey\":\"hex\",\"redeemScript\":\"hex\",\"amount\":value},...] [\"privatekey1\",...] sighashtype )");
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    const CChainParams& params = cs.Params();
    std::vector<unsigned char> txData(ParseHexV(req.params[0], "argument 1"));
    std::vector<CMutableTransaction> txVariants;
    {
        SpanReader r(txData.data(), txData.size());
        while (!r.empty()) {
            try {
                CMutableTransaction tx;
                r >> tx;
                txVariants.push_back(tx);
            } catch (const std::exception&) {
                ThrowRPC(RPC_DESERIALIZATION_ERROR, "TX decode failed");
            }
        }
    }
    if (txVariants.empty()) ThrowRPC(RPC_DESERIALIZATION_ERROR, "Missing transaction");
    CMutableTransaction mergedTx(txVariants[0]);
    CCoinsView viewDummy;
    CCoinsViewCache view(&viewDummy);
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        std::lock_guard<CCriticalSection> lm(n.mempool->cs);
        CCoinsViewCache& viewChain = cs.CoinsTip();
        CCoinsViewMemPool viewMempool(&viewChain, *n.mempool);
        view.SetBackend(viewMempool);
        for (const CTxIn& txin : mergedTx.vin) view.AccessCoin(txin.prevout); // load into cache
        view.SetBackend(viewDummy);
    }
    bool fGivenKeys = false;
    CBasicKeyStore tempKeystore;
    if (req.params.size() > 2 && !req.params[2].isNull()) {
        fGivenKeys = true;
        const UniValue& keys = req.params[2].get_array();
        for (size_t idx = 0; idx < keys.size(); idx++) {
            CKey key = DecodeSecret(keys[idx].get_str(), params);
            if (!key.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid private key");
            tempKeystore.AddKey(key);
        }
    }
    if (req.params.size() > 1 && !req.params[1].isNull()) {
        const UniValue& prevTxs = req.params[1].get_array();
        for (size_t idx = 0; idx < prevTxs.size(); idx++) {
            const UniValue& p = prevTxs[idx];
            if (!p.isObject()) ThrowRPC(RPC_DESERIALIZATION_ERROR, "expected object with {\"txid'\",\"vout\",\"scriptPubKey\"}");
            const uint256 txid = ParseHashO(p, "txid");
            if (!p["vout"].isNum()) ThrowRPC(RPC_TYPE_ERROR, "Missing vout");
            const int nOut = p["vout"].get_int();
            if (nOut < 0) ThrowRPC(RPC_DESERIALIZATION_ERROR, "vout must be positive");
            const COutPoint out(txid, (uint32_t)nOut);
            std::vector<unsigned char> pkData(ParseHexO(p, "scriptPubKey"));
            CScript scriptPubKey(pkData.begin(), pkData.end());
            const Coin& coin = view.AccessCoin(out);
            if (!coin.IsSpent() && coin.GetTxOut().scriptPubKey != scriptPubKey)
                ThrowRPC(RPC_DESERIALIZATION_ERROR, "Previous output scriptPubKey mismatch:\n" +
                                                       ScriptToAsmStr(coin.GetTxOut().scriptPubKey) + "\nvs:\n" +
                                                       ScriptToAsmStr(scriptPubKey));
            CTxOut txout;
            txout.scriptPubKey = scriptPubKey;
            txout.nValue = 0;
            if (p.exists("amount")) txout.nValue = AmountFromValue(p["amount"]);
            else ThrowRPC(RPC_INVALID_PARAMETER, "Missing amount");
            view.AddCoin(out, Coin(txout, 1, false), true);
            if (fGivenKeys && scriptPubKey.IsPayToScriptHash()) {
                const UniValue& v = p["redeemScript"];
                if (!v.isNull()) {
                    std::vector<unsigned char> rsData(ParseHexV(v, "redeemScript"));
                    tempKeystore.AddCScript(CScript(rsData.begin(), rsData.end()));
                }
            }
        }
    }
    const CKeyStore& keystore = (fGivenKeys || !n.keystore) ? static_cast<const CKeyStore&>(tempKeystore) : *n.keystore;
    int nHashType = SIGHASH_ALL | SIGHASH_FORKID;
    if (req.params.size() > 3 && !req.params[3].isNull()) {
        nHashType = ParseSighashString(req.params[3].get_str());
        if ((nHashType & SIGHASH_FORKID) == 0) ThrowRPC(RPC_INVALID_PARAMETER, "Signature must use SIGHASH_FORKID");
    }
    const bool fHashSingle = ((nHashType & ~(SIGHASH_ANYONECANPAY | SIGHASH_FORKID)) == SIGHASH_SINGLE);
    UniValue vErrors(UniValue::VARR);
    const CTransaction txConst(mergedTx);
    for (size_t i = 0; i < mergedTx.vin.size(); i++) {
        CTxIn& txin = mergedTx.vin[i];
        const Coin& coin = view.AccessCoin(txin.prevout);
        if (coin.IsSpent()) {
            TxInErrorToJSON(txin, vErrors, "Input not found or already spent");
            continue;
        }
        const CScript& prevPubKey = coin.GetTxOut().scriptPubKey;
        const Amount amount = coin.GetTxOut().nValue;
        SignatureData sigdata;
        if (!fHashSingle || i < mergedTx.vout.size()) {
            TransactionSignatureCreator creator(&keystore, &txConst, (unsigned)i, amount, (uint32_t)nHashType);
            ProduceSignature(creator, prevPubKey, sigdata);
        }
        for (const CMutableTransaction& txv : txVariants)
            if (txv.vin.size() > i)
                sigdata = CombineSignatures(prevPubKey, TransactionSignatureChecker(&txConst, (unsigned)i, amount), sigdata,
                                            DataFromTransaction(txv, (unsigned)i));
        UpdateTransaction(mergedTx, (unsigned)i, sigdata);
        ScriptError serror = SCRIPT_ERR_OK;
        if (!VerifyScript(txin.scriptSig, prevPubKey, STANDARD_SCRIPT_VERIFY_FLAGS,
                          TransactionSignatureChecker(&txConst, (unsigned)i, amount), &serror))
            TxInErrorToJSON(txin, vErrors, ScriptErrorString(serror));
    }
    UniValue result(UniValue::VOBJ);
    result.pushKV("hex", EncodeHexTx(CTransaction(mergedTx)));
    result.pushKV("complete", vErrors.empty());
    if (!vErrors.empty()) result.pushKV("errors", vErrors);
    return result;
}

static UniValue sendrawtransaction(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "sendrawtransaction \"hexstring\" ( allowhighfees )");
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    CMutableTransaction mtx;
    if (!DecodeHexTx(mtx, req.params[0].get_str())) ThrowRPC(RPC_DESERIALIZATION_ERROR, "TX decode failed");
    CTransactionRef tx(MakeTransactionRef(std::move(mtx)));
    const uint256& txid = tx->GetHash();
    Amount nMaxRawTxFee = DEFAULT_TRANSACTION_MAXFEE;
    if (req.params.size() > 1 && !req.params[1].isNull() && req.params[1].get_bool()) nMaxRawTxFee = 0;
    bool fHaveChain = false;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        for (size_t o = 0; !fHaveChain && o < tx->vout.size(); o++)
            fHaveChain = !cs.CoinsTip().AccessCoin(COutPoint(txid, (uint32_t)o)).IsSpent();
    }
    const bool fHaveMempool = n.mempool->exists(txid);
    if (!fHaveMempool && !fHaveChain) {
        CValidationState state;
        bool fMissingInputs = false;
        if (!cs.AcceptToMemoryPool(state, tx, false, &fMissingInputs, false, nMaxRawTxFee)) {
            if (state.IsInvalid())
                ThrowRPC(RPC_TRANSACTION_REJECTED, strprintf("%i: %s", state.GetRejectCode(), state.GetRejectReason().c_str()));
            if (fMissingInputs) ThrowRPC(RPC_TRANSACTION_ERROR, "Missing inputs");
            ThrowRPC(RPC_TRANSACTION_ERROR, state.GetRejectReason());
        }
    } else if (fHaveChain) {
        ThrowRPC(RPC_TRANSACTION_ALREADY_IN_CHAIN, "transaction already in block chain");
    }
    if (g_relayTransaction) g_relayTransaction(txid);
    return txid.GetHex();
}

static UniValue gettxoutproof(const JSONRPCRequest& req) {
    if (req.params.size() != 1 && req.params.size() != 2)
        ThrowRPC(RPC_INVALID_PARAMS, "gettxoutproof [\"txid\",...] ( blockhash )");
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::set<uint256> setTxids;
    uint256 oneTxid;
    const UniValue& txids = req.params[0].get_array();
    for (size_t idx = 0; idx < txids.size(); idx++) {
        const std::string& txid = txids[idx].get_str();
        if (txid.size() != 64 || !IsHex(txid)) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid txid " + txid);
        const uint256 hash = uint256S(txid);
        if (setTxids.count(hash)) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated txid: " + txid);
        setTxids.insert(hash);
        oneTxid = hash;
    }
    std::lock_guard<CCriticalSection> l(cs.cs());
    CBlockIndex* pblockindex = nullptr;
    uint256 hashBlock;
    if (req.params.size() > 1) {
        hashBlock = uint256S(req.params[1].get_str());
        pblockindex = cs.LookupBlockIndex(hashBlock);
        if (!pblockindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
    } else {
        const Coin& coin = AccessByTxid(cs.CoinsTip(), oneTxid);
        if (!coin.IsSpent() && coin.GetHeight() > 0 && (int)coin.GetHeight() <= cs.Height())
            pblockindex = cs.ActiveChain()[coin.GetHeight()];
    }
    if (pblockindex == nullptr) {
        CTransactionRef tx;
        if (!cs.GetTransaction(oneTxid, tx, hashBlock, false) || hashBlock.IsNull())
            ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not yet in block");
        pblockindex = cs.LookupBlockIndex(hashBlock);
        if (!pblockindex) ThrowRPC(RPC_INTERNAL_ERROR, "Transaction index corrupt");
    }
    CBlock block;
    if (!cs.ReadBlock(block, pblockindex)) ThrowRPC(RPC_INTERNAL_ERROR, "Can't read block from disk");
    unsigned ntxFound = 0;
    for (const auto& tx : block.vtx)
        if (setTxids.count(tx->GetHash())) ntxFound++;
    if (ntxFound != setTxids.size()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "(Not all) transactions not found in specified block");
    CMerkleBlock mb(block, setTxids);
    const bool legacy = pblockindex->nHeight < cs.Params().GetConsensus().BCPHeight;
    return HexStr(SerializeToBytes(mb, SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0)));
}

static UniValue verifytxoutproof(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "verifytxoutproof \"proof\"");
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::vector<unsigned char> data = ParseHexV(req.params[0], "proof");
    CMerkleBlock merkleBlock;
    if (!DecodeTxOutProof(data, merkleBlock)) ThrowRPC(RPC_DESERIALIZATION_ERROR, "Proof decode failed");
    UniValue res(UniValue::VARR);
    std::vector<uint256> vMatch;
    std::vector<unsigned> vIndex;
    if (merkleBlock.txn.ExtractMatches(vMatch, vIndex) != merkleBlock.header.hashMerkleRoot) return res;
    std::lock_guard<CCriticalSection> l(cs.cs());
    CBlockIndex* pindex = cs.LookupBlockIndex(merkleBlock.header.GetHash(cs.Params().GetConsensus()));
    if (!pindex || !cs.ActiveChain().Contains(pindex)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found in chain");
    for (const uint256& h : vMatch) res.push_back(h.GetHex());
    return res;
}

void RegisterRawTransactionRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"rawtransactions", "getrawtransaction", getrawtransaction, true, {"txid", "verbose"}, "getrawtransaction \"txid\" ( verbose )\nReturn the raw transaction data."},
        {"rawtransactions", "createrawtransaction", createrawtransaction, true, {"inputs", "outputs", "locktime"}, "createrawtransaction [{\"txid\":\"id\",\"vout\":n},...] {\"address\":amount,\"data\":\"hex\",...} ( locktime )\nCreate a transaction spending the given inputs and creating new outputs."},
        {"rawtransactions", "decoderawtransaction", decoderawtransaction, true, {"hexstring"}, "decoderawtransaction \"hexstring\"\nReturn a JSON object representing the serialized, hex-encoded transaction."},
        {"rawtransactions", "decodescript", decodescript, true, {"hexstring"}, "decodescript \"hexstring\"\nDecode a hex-encoded script."},
        {"rawtransactions", "sendrawtransaction", sendrawtransaction, false, {"hexstring", "allowhighfees"}, "sendrawtransaction \"hexstring\" ( allowhighfees )\nSubmits raw transaction (serialized, hex-encoded) to local node and network."},
        {"rawtransactions", "signrawtransaction", signrawtransaction, false, {"hexstring", "prevtxs", "privkeys", "sighashtype"}, "signrawtransaction \"hexstring\" ( [{\"txid\":\"id\",\"vout\":n,\"scriptPubKey\":\"hex\",\"redeemScript\":\"hex\",\"amount\":value},...] [\"privatekey1\",...] sighashtype )\nSign inputs for raw transaction (FORKID signatures)."},
        {"blockchain", "gettxoutproof", gettxoutproof, true, {"txids", "blockhash"}, "gettxoutproof [\"txid\",...] ( blockhash )\nReturns a hex-encoded proof that \"txid\" was included in a block."},
        {"blockchain", "verifytxoutproof", verifytxoutproof, true, {"proof"}, "verifytxoutproof \"proof\"\nVerifies that a proof points to a transaction in a block."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
