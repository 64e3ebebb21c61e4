// Blockchain RPCs. Parity: reference src/rpc/blockchain.cpp (command table :1646;
// blockheaderToJSON/blockToJSON :68-160 incl. BCP fields nonce (256-bit hex),
// nonceUint32 and solution; getblock verbosity + `legacy` serialization flag).
#include "consensus/merkle.h"
#include "node/node.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "rpc/core_io.h"
#include "rpc/server.h"
#include "util/strencodings.h"

#include <cmath>

namespace bcp {

static NodeContext& Node() {
    NodeContext* n = GetNode();
    if (!n || !n->chainstate) ThrowRPC(RPC_INTERNAL_ERROR, "node not initialised");
    return *n;
}

double GetDifficulty(const CBlockIndex* blockindex) {
    if (blockindex == nullptr) return 1.0;
    return GetDifficultyFromBits(blockindex->nBits);
}

UniValue blockheaderToJSON(const CBlockIndex* blockindex) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs()); // confirmations / next block read the active chain
    UniValue result(UniValue::VOBJ);
    result.pushKV("hash", blockindex->GetBlockHash().GetHex());
    int confirmations = -1;
    if (cs.ActiveChain().Contains(blockindex)) confirmations = cs.Height() - blockindex->nHeight + 1;
    result.pushKV("confirmations", confirmations);
    result.pushKV("height", blockindex->nHeight);
    result.pushKV("version", blockindex->nVersion);
    result.pushKV("versionHex", strprintf("%08x", blockindex->nVersion));
    result.pushKV("merkleroot", blockindex->hashMerkleRoot.GetHex());
    result.pushKV("time", (int64_t)blockindex->nTime);
    result.pushKV("mediantime", (int64_t)blockindex->GetMedianTimePast());
    result.pushKV("nonceUint32", (uint64_t)(uint32_t)blockindex->nNonce.GetUint64(0));
    result.pushKV("nonce", blockindex->nNonce.GetHex());
    result.pushKV("solution", HexStr(blockindex->nSolution));
    result.pushKV("bits", strprintf("%08x", blockindex->nBits));
    result.pushKV("difficulty", GetDifficulty(blockindex));
    result.pushKV("chainwork", blockindex->nChainWork.GetHex());
    if (blockindex->pprev) result.pushKV("previousblockhash", blockindex->pprev->GetBlockHash().GetHex());
    if (CBlockIndex* pnext = cs.ActiveChain().Next(blockindex)) result.pushKV("nextblockhash", pnext->GetBlockHash().GetHex());
    return result;
}

UniValue blockToJSON(const CBlock& block, const CBlockIndex* blockindex, bool txDetails) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const CChainParams& params = cs.Params();
    UniValue result(UniValue::VOBJ);
    result.pushKV("hash", blockindex->GetBlockHash().GetHex());
    int confirmations = -1;
    if (cs.ActiveChain().Contains(blockindex)) confirmations = cs.Height() - blockindex->nHeight + 1;
    result.pushKV("confirmations", confirmations);
    const int serFlags = blockindex->nHeight < params.GetConsensus().BCPHeight ? SERIALIZE_BLOCK_LEGACY : 0;
    result.pushKV("size", (int)GetSerializeSize(block, PROTOCOL_VERSION | serFlags));
    result.pushKV("height", blockindex->nHeight);
    result.pushKV("version", block.nVersion);
    result.pushKV("versionHex", strprintf("%08x", block.nVersion));
    result.pushKV("merkleroot", block.hashMerkleRoot.GetHex());
    UniValue txs(UniValue::VARR);
    for (const auto& tx : block.vtx) {
        if (txDetails) {
            UniValue objTx(UniValue::VOBJ);
            TxToUniv(*tx, uint256(), objTx, params);
            txs.push_back(objTx);
        } else {
            txs.push_back(tx->GetHash().GetHex());
        }
    }
    result.pushKV("tx", txs);
    result.pushKV("time", block.GetBlockTime());
    result.pushKV("mediantime", (int64_t)blockindex->GetMedianTimePast());
    result.pushKV("nonceUint32", (uint64_t)(uint32_t)blockindex->nNonce.GetUint64(0));
    result.pushKV("nonce", blockindex->nNonce.GetHex());
    result.pushKV("solution", HexStr(block.nSolution));
    result.pushKV("bits", strprintf("%08x", block.nBits));
    result.pushKV("difficulty", GetDifficulty(blockindex));
    result.pushKV("chainwork", blockindex->nChainWork.GetHex());
    if (blockindex->pprev) result.pushKV("previousblockhash", blockindex->pprev->GetBlockHash().GetHex());
    if (CBlockIndex* pnext = cs.ActiveChain().Next(blockindex)) result.pushKV("nextblockhash", pnext->GetBlockHash().GetHex());
    return result;
}

static UniValue getblockcount(const JSONRPCRequest& req) {
    if (req.params.size() != 0) ThrowRPC(RPC_INVALID_PARAMS, "getblockcount takes no arguments");
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    return cs.Height();
}

static UniValue getbestblockhash(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    return cs.Tip()->GetBlockHash().GetHex();
}

static UniValue getdifficulty(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    return GetDifficulty(cs.Tip());
}

static UniValue getblockhash(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "getblockhash height");
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const int nHeight = req.params[0].get_int();
    if (nHeight < 0 || nHeight > cs.Height()) ThrowRPC(RPC_INVALID_PARAMETER, "Block height out of range");
    return cs.ActiveChain()[nHeight]->GetBlockHash().GetHex();
}

static UniValue getblockheader(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "getblockheader \"hash\" ( verbose )");
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const uint256 hash = uint256S(req.params[0].get_str());
    const bool fVerbose = req.params.size() > 1 && !req.params[1].isNull() ? req.params[1].get_bool() : true;
    CBlockIndex* pblockindex = cs.LookupBlockIndex(hash);
    if (!pblockindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
    if (!fVerbose) {
        const CBlockHeader h = pblockindex->GetBlockHeader();
        const bool legacy = pblockindex->nHeight < cs.Params().GetConsensus().BCPHeight;
        return HexStr(SerializeToBytes(h, SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0)));
    }
    return blockheaderToJSON(pblockindex);
}

static UniValue getblock(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "getblock \"blockhash\" ( verbose legacy )");
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const uint256 hash = uint256S(req.params[0].get_str());
    int verbosity = 1;
    if (req.params.size() > 1 && !req.params[1].isNull())
        verbosity = req.params[1].isNum() ? req.params[1].get_int() : (req.params[1].get_bool() ? 1 : 0);
    const bool legacy = req.params.size() > 2 && !req.params[2].isNull() && req.params[2].get_bool();
    CBlockIndex* pblockindex = cs.LookupBlockIndex(hash);
    if (!pblockindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
    if (cs.HavePruned() && !(pblockindex->nStatus & BLOCK_HAVE_DATA) && pblockindex->nTx > 0)
        ThrowRPC(RPC_MISC_ERROR, "Block not available (pruned data)");
    CBlock block;
    if (!cs.ReadBlock(block, pblockindex)) ThrowRPC(RPC_MISC_ERROR, "Can't read block from disk");
    if (verbosity <= 0) return EncodeHexBlock(block, legacy);
    return blockToJSON(block, pblockindex, verbosity >= 2);
}

static UniValue getchaintips(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    UniValue res(UniValue::VARR);
    for (const CBlockIndex* block : cs.GetChainTips()) {
        UniValue obj(UniValue::VOBJ);
        obj.pushKV("height", block->nHeight);
        obj.pushKV("hash", block->phashBlock->GetHex());
        const int branchLen = block->nHeight - cs.ActiveChain().FindFork(block)->nHeight;
        obj.pushKV("branchlen", branchLen);
        std::string status;
        if (cs.ActiveChain().Contains(block)) status = "active";
        else if (block->nStatus & BLOCK_FAILED_MASK) status = "invalid";
        else if (block->nChainTx == 0) status = "headers-only";
        else if (block->IsValid(BLOCK_VALID_SCRIPTS)) status = "valid-fork";
        else if (block->IsValid(BLOCK_VALID_TREE)) status = "valid-headers";
        else status = "unknown";
        obj.pushKV("status", status);
        res.push_back(obj);
    }
    return res;
}

static UniValue BIP9SoftForkDesc(Chainstate& cs, Consensus::DeploymentPos id) EXCLUSIVE_LOCKS_REQUIRED(cs.cs()) {
    UniValue rv(UniValue::VOBJ);
    const ThresholdState st = cs.DeploymentState(cs.Tip(), id);
    rv.pushKV("status", ThresholdStateName(st));
    if (st == THRESHOLD_STARTED) rv.pushKV("bit", cs.Params().GetConsensus().vDeployments[id].bit);
    rv.pushKV("startTime", cs.Params().GetConsensus().vDeployments[id].nStartTime);
    rv.pushKV("timeout", cs.Params().GetConsensus().vDeployments[id].nTimeout);
    rv.pushKV("since", VersionBitsStateSinceHeight(cs.Tip(), cs.Params().GetConsensus(), id, cs.VersionBits()));
    return rv;
}

static UniValue SoftForkDesc(const std::string& name, int version, const CBlockIndex* pindex, const Consensus::Params& cp) {
    UniValue rv(UniValue::VOBJ);
    rv.pushKV("id", name);
    rv.pushKV("version", version);
    bool active = false;
    if (name == "bip34") active = pindex->nHeight >= cp.BIP34Height;
    else if (name == "bip66") active = pindex->nHeight >= cp.BIP66Height;
    else if (name == "bip65") active = pindex->nHeight >= cp.BIP65Height;
    UniValue r(UniValue::VOBJ);
    r.pushKV("status", active);
    rv.pushKV("reject", r);
    return rv;
}

static UniValue getblockchaininfo(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const Consensus::Params& cp = cs.Params().GetConsensus();
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("chain", cs.Params().NetworkIDString());
    obj.pushKV("blocks", cs.Height());
    obj.pushKV("headers", cs.BestHeader() ? cs.BestHeader()->nHeight : -1);
    obj.pushKV("bestblockhash", cs.Tip()->GetBlockHash().GetHex());
    obj.pushKV("difficulty", GetDifficulty(cs.Tip()));
    obj.pushKV("mediantime", (int64_t)cs.Tip()->GetMedianTimePast());
    obj.pushKV("verificationprogress", cs.GuessVerificationProgress(cs.Tip()));
    obj.pushKV("chainwork", cs.Tip()->nChainWork.GetHex());
    obj.pushKV("pruned", cs.PruneMode());
    obj.pushKV("bcpheight", cp.BCPHeight);
    obj.pushKV("equihash", strprintf("%u,%u", cs.Params().EquihashN(), cs.Params().EquihashK()));
    UniValue softforks(UniValue::VARR);
    softforks.push_back(SoftForkDesc("bip34", 2, cs.Tip(), cp));
    softforks.push_back(SoftForkDesc("bip66", 3, cs.Tip(), cp));
    softforks.push_back(SoftForkDesc("bip65", 4, cs.Tip(), cp));
    UniValue bip9(UniValue::VOBJ);
    bip9.pushKV("csv", BIP9SoftForkDesc(cs, Consensus::DEPLOYMENT_CSV));
    obj.pushKV("softforks", softforks);
    obj.pushKV("bip9_softforks", bip9);
    if (cs.PruneMode()) {
        const CBlockIndex* block = cs.Tip();
        while (block && block->pprev && (block->pprev->nStatus & BLOCK_HAVE_DATA)) block = block->pprev;
        obj.pushKV("pruneheight", block ? block->nHeight : 0);
    }
    obj.pushKV("warnings", cs.Warnings());
    return obj;
}

// ---- mempool
static UniValue entryToJSON(const CTxMemPoolEntry& e, CTxMemPool& pool, int height) {
    UniValue info(UniValue::VOBJ);
    info.pushKV("size", (int)e.GetTxSize());
    info.pushKV("fee", ValueFromAmount(e.GetFee()));
    info.pushKV("modifiedfee", ValueFromAmount(e.GetModifiedFee()));
    info.pushKV("time", e.GetTime());
    info.pushKV("height", (int)e.GetHeight());
    info.pushKV("startingpriority", e.GetPriority(e.GetHeight()));
    info.pushKV("currentpriority", e.GetPriority(height));
    info.pushKV("descendantcount", e.GetCountWithDescendants());
    info.pushKV("descendantsize", e.GetSizeWithDescendants());
    info.pushKV("descendantfees", e.GetModFeesWithDescendants());
    info.pushKV("ancestorcount", e.GetCountWithAncestors());
    info.pushKV("ancestorsize", e.GetSizeWithAncestors());
    info.pushKV("ancestorfees", e.GetModFeesWithAncestors());
    UniValue depends(UniValue::VARR);
    std::set<std::string> setDepends;
    for (const CTxIn& in : e.GetTx().vin)
        if (pool.exists(in.prevout.hash)) setDepends.insert(in.prevout.hash.ToString());
    for (const std::string& d : setDepends) depends.push_back(d);
    info.pushKV("depends", depends);
    return info;
}

UniValue mempoolToJSON(bool fVerbose) {
    NodeContext& n = Node();
    CTxMemPool& pool = *n.mempool;
    if (fVerbose) {
        const int height = n.chainstate->HeightNow(); // before the mempool lock: cs_main comes first
        std::lock_guard<CCriticalSection> l(pool.cs);
        UniValue o(UniValue::VOBJ);
        for (const CTxMemPoolEntry* e : pool.SortedByDepthAndScore())
            o.pushKV(e->GetTx().GetHash().ToString(), entryToJSON(*e, pool, height));
        return o;
    }
    std::vector<uint256> vtxid;
    pool.queryHashes(vtxid);
    UniValue a(UniValue::VARR);
    for (const uint256& h : vtxid) a.push_back(h.ToString());
    return a;
}

static UniValue getrawmempool(const JSONRPCRequest& req) {
    bool fVerbose = req.params.size() > 0 && !req.params[0].isNull() && req.params[0].get_bool();
    return mempoolToJSON(fVerbose);
}

static UniValue mempoolRelatives(const JSONRPCRequest& req, bool ancestors) {
    NodeContext& n = Node();
    const uint256 hash = ParseHashV(req.params[0], "parameter 1");
    const bool fVerbose = req.params.size() > 1 && !req.params[1].isNull() && req.params[1].get_bool();
    const int height = n.chainstate->HeightNow(); // before the mempool lock: cs_main comes first
    std::lock_guard<CCriticalSection> l(n.mempool->cs);
    if (!n.mempool->exists(hash)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not in mempool");
    auto rel = ancestors ? n.mempool->GetAncestors(hash) : n.mempool->GetDescendants(hash);
    if (!fVerbose) {
        UniValue o(UniValue::VARR);
        for (const auto* e : rel) o.push_back(e->GetTx().GetHash().ToString());
        return o;
    }
    UniValue o(UniValue::VOBJ);
    for (const auto* e : rel) o.pushKV(e->GetTx().GetHash().ToString(), entryToJSON(*e, *n.mempool, height));
    return o;
}
static UniValue getmempoolancestors(const JSONRPCRequest& req) { return mempoolRelatives(req, true); }
static UniValue getmempooldescendants(const JSONRPCRequest& req) { return mempoolRelatives(req, false); }

static UniValue getmempoolentry(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    const uint256 hash = ParseHashV(req.params[0], "parameter 1");
    const int height = n.chainstate->HeightNow();
    std::lock_guard<CCriticalSection> l(n.mempool->cs);
    const CTxMemPoolEntry* e = n.mempool->GetEntry(hash);
    if (!e) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not in mempool");
    return entryToJSON(*e, *n.mempool, height);
}

UniValue mempoolInfoToJSON() {
    NodeContext& n = Node();
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("size", (int64_t)n.mempool->size());
    ret.pushKV("bytes", (int64_t)n.mempool->GetTotalTxSize());
    ret.pushKV("usage", (int64_t)n.mempool->DynamicMemoryUsage());
    const size_t maxmempool = (size_t)gArgs.GetArg("-maxmempool", (int64_t)300) * 1000000;
    ret.pushKV("maxmempool", (int64_t)maxmempool);
    ret.pushKV("mempoolminfee", ValueFromAmount(n.mempool->GetMinFee(maxmempool).GetFeePerK()));
    return ret;
}
static UniValue getmempoolinfo(const JSONRPCRequest& req) { return mempoolInfoToJSON(); }

// ---- UTXO
static UniValue gettxout(const JSONRPCRequest& req) {
    if (req.params.size() < 2 || req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "gettxout \"txid\" n ( include_mempool )");
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const uint256 hash = ParseHashV(req.params[0], "txid");
    const COutPoint out(hash, (uint32_t)req.params[1].get_int());
    const bool fMempool = req.params.size() > 2 && !req.params[2].isNull() ? req.params[2].get_bool() : true;
    Coin coin;
    if (fMempool) {
        std::lock_guard<CCriticalSection> lm(n.mempool->cs);
        CCoinsViewMemPool view(&cs.CoinsTip(), *n.mempool);
        if (!view.GetCoin(out, coin) || n.mempool->isSpent(out)) return UniValue::NullUniValue;
    } else {
        if (!cs.CoinsTip().GetCoin(out, coin) || coin.IsSpent()) return UniValue::NullUniValue;
    }
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("bestblock", cs.Tip()->GetBlockHash().GetHex());
    if (coin.GetHeight() == MEMPOOL_HEIGHT) ret.pushKV("confirmations", 0);
    else ret.pushKV("confirmations", (int64_t)(cs.Height() - coin.GetHeight() + 1));
    ret.pushKV("value", ValueFromAmount(coin.GetTxOut().nValue));
    UniValue o(UniValue::VOBJ);
    ScriptPubKeyToUniv(coin.GetTxOut().scriptPubKey, o, true, cs.Params());
    ret.pushKV("scriptPubKey", o);
    ret.pushKV("coinbase", coin.IsCoinBase());
    return ret;
}

static UniValue gettxoutsetinfo(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    cs.FlushStateToDisk();
    std::unique_ptr<CCoinsViewCursor> pcursor = cs.CoinsDB().Cursor();
    HashWriter ss;
    ss << pcursor->GetBestBlock();
    uint64_t nTransactions = 0, nTransactionOutputs = 0, nBogoSize = 0;
    Amount nTotalAmount = 0;
    uint256 prevkey;
    std::map<uint32_t, Coin> outputs;
    auto flushTx = [&](const uint256& hash) {
        if (outputs.empty()) return;
        nTransactions++;
        ss << hash;
        ss << VARINT(outputs.begin()->second.nHeight * 2 + (outputs.begin()->second.fCoinBase ? 1 : 0));
        for (const auto& o : outputs) {
            ss << VARINT(o.first + 1);
            ss << o.second.out.scriptPubKey;
            ss << VARINT((uint64_t)o.second.out.nValue);
            nTransactionOutputs++;
            nTotalAmount += o.second.out.nValue;
            nBogoSize += 32 + 4 + 4 + 8 + 2 + o.second.out.scriptPubKey.size(); // txid, n, height, value, script length
        }
        ss << VARINT(0u);
        outputs.clear();
    };
    while (pcursor->Valid()) {
        COutPoint key;
        Coin coin;
        if (pcursor->GetKey(key) && pcursor->GetValue(coin)) {
            if (!outputs.empty() && key.hash != prevkey) flushTx(prevkey);
            prevkey = key.hash;
            outputs[key.n] = std::move(coin);
        }
        pcursor->Next();
    }
    flushTx(prevkey);
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("height", cs.Height());
    ret.pushKV("bestblock", cs.Tip()->GetBlockHash().GetHex());
    ret.pushKV("transactions", (int64_t)nTransactions);
    ret.pushKV("txouts", (int64_t)nTransactionOutputs);
    ret.pushKV("bogosize", (int64_t)nBogoSize);
    ret.pushKV("hash_serialized", ss.GetHash().GetHex());
    ret.pushKV("disk_size", (int64_t)cs.CoinsDB().EstimateSize());
    ret.pushKV("total_amount", ValueFromAmount(nTotalAmount));
    return ret;
}

static UniValue verifychain(const JSONRPCRequest& req) {
    int nCheckLevel = (int)gArgs.GetArg("-checklevel", (int64_t)DEFAULT_CHECKLEVEL);
    int nCheckDepth = (int)gArgs.GetArg("-checkblocks", (int64_t)DEFAULT_CHECKBLOCKS);
    if (req.params.size() > 0 && !req.params[0].isNull()) nCheckLevel = req.params[0].get_int();
    if (req.params.size() > 1 && !req.params[1].isNull()) nCheckDepth = req.params[1].get_int();
    return Node().chainstate->VerifyDB(nCheckLevel, nCheckDepth);
}

static UniValue preciousblock(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    const uint256 hash = uint256S(req.params[0].get_str());
    CBlockIndex* pindex;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        pindex = cs.LookupBlockIndex(hash);
        if (!pindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
    }
    CValidationState state;
    cs.PreciousBlock(state, pindex);
    if (!state.IsValid()) ThrowRPC(RPC_DATABASE_ERROR, state.GetRejectReason());
    return UniValue::NullUniValue;
}

static UniValue invalidateblock(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    const uint256 hash = uint256S(req.params[0].get_str());
    CValidationState state;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        CBlockIndex* pindex = cs.LookupBlockIndex(hash);
        if (!pindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
        cs.InvalidateBlock(state, pindex);
    }
    if (state.IsValid()) cs.ActivateBestChain(state);
    if (!state.IsValid()) ThrowRPC(RPC_DATABASE_ERROR, state.GetRejectReason());
    return UniValue::NullUniValue;
}

static UniValue reconsiderblock(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    const uint256 hash = uint256S(req.params[0].get_str());
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        CBlockIndex* pindex = cs.LookupBlockIndex(hash);
        if (!pindex) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found");
        cs.ResetBlockFailureFlags(pindex);
    }
    CValidationState state;
    cs.ActivateBestChain(state);
    if (!state.IsValid()) ThrowRPC(RPC_DATABASE_ERROR, state.GetRejectReason());
    return UniValue::NullUniValue;
}

static UniValue pruneblockchain(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    if (!cs.PruneMode()) ThrowRPC(RPC_MISC_ERROR, "Cannot prune blocks because node is not in prune mode.");
    std::lock_guard<CCriticalSection> l(cs.cs());
    int heightParam = req.params[0].get_int();
    if (heightParam < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Negative block height.");
    if (heightParam > 1000000000) {
        // a timestamp: prune to the last block at or before it
        CBlockIndex* pindex = cs.ActiveChain().FindEarliestAtLeast(heightParam);
        if (!pindex) ThrowRPC(RPC_INVALID_PARAMETER, "Could not find block with at least the specified timestamp.");
        heightParam = pindex->nHeight;
    }
    const unsigned h = (unsigned)heightParam;
    unsigned chainHeight = (unsigned)cs.Height();
    if (chainHeight < cs.Params().PruneAfterHeight()) ThrowRPC(RPC_MISC_ERROR, "Blockchain is too short for pruning.");
    if (h > chainHeight) ThrowRPC(RPC_INVALID_PARAMETER, "Blockchain is shorter than the attempted prune height.");
    const unsigned height = std::min(h, chainHeight - MIN_BLOCKS_TO_KEEP);
    cs.PruneBlockFilesManual((int)height);
    return (uint64_t)height;
}

static UniValue waitforblockimpl(const JSONRPCRequest& req, const uint256* target, int targetHeight) {
    Chainstate& cs = *Node().chainstate;
    int timeout = 0;
    const size_t idx = (target || targetHeight >= 0) ? 1 : 0;
    if (req.params.size() > idx && !req.params[idx].isNull()) timeout = req.params[idx].get_int();
    const int64_t deadline = GetTimeMillis() + timeout;
    std::unique_lock<CCriticalSection> l(cs.cs());
    AssertLockHeld(cs.cs()); // (unique_lock is invisible to the thread-safety analysis)
    const uint256 start = cs.Tip()->GetBlockHash();
    auto done = [&] {
        AssertLockHeld(cs.cs()); // evaluated with `l` held
        if (ShutdownRequested()) return true;
        if (target) return cs.Tip()->GetBlockHash() == *target;
        if (targetHeight >= 0) return cs.Height() >= targetHeight;
        return cs.Tip()->GetBlockHash() != start;
    };
    while (!done()) {
        if (timeout) {
            const int64_t left = deadline - GetTimeMillis();
            if (left <= 0) break;
            cs.BlockChangeCV().wait_for(l, std::chrono::milliseconds(std::min<int64_t>(left, 1000)));
        } else {
            cs.BlockChangeCV().wait_for(l, std::chrono::milliseconds(1000));
        }
    }
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("hash", cs.Tip()->GetBlockHash().GetHex());
    ret.pushKV("height", cs.Height());
    return ret;
}
static UniValue waitfornewblock(const JSONRPCRequest& req) { return waitforblockimpl(req, nullptr, -1); }
static UniValue waitforblock(const JSONRPCRequest& req) {
    const uint256 h = uint256S(req.params[0].get_str());
    return waitforblockimpl(req, &h, -1);
}
static UniValue waitforblockheight(const JSONRPCRequest& req) { return waitforblockimpl(req, nullptr, req.params[0].get_int()); }

void RegisterBlockchainRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"blockchain", "getblockchaininfo", getblockchaininfo, true, {}, "getblockchaininfo\nReturns an object containing various state info regarding blockchain processing."},
        {"blockchain", "getbestblockhash", getbestblockhash, true, {}, "getbestblockhash\nReturns the hash of the best (tip) block in the longest blockchain."},
        {"blockchain", "getblockcount", getblockcount, true, {}, "getblockcount\nReturns the number of blocks in the longest blockchain."},
        {"blockchain", "getblock", getblock, true, {"blockhash", "verbose", "legacy"}, "getblock \"blockhash\" ( verbose legacy )\nReturns block data; verbose=0 hex (legacy=true for the 80-byte header format)."},
        {"blockchain", "getblockhash", getblockhash, true, {"height"}, "getblockhash height\nReturns hash of block in best-block-chain at height provided."},
        {"blockchain", "getblockheader", getblockheader, true, {"blockhash", "verbose"}, "getblockheader \"hash\" ( verbose )\nReturns information about a block header."},
        {"blockchain", "getchaintips", getchaintips, true, {}, "getchaintips\nReturn information about all known tips in the block tree."},
        {"blockchain", "getdifficulty", getdifficulty, true, {}, "getdifficulty\nReturns the proof-of-work difficulty as a multiple of the minimum difficulty."},
        {"blockchain", "getmempoolancestors", getmempoolancestors, true, {"txid", "verbose"}, "getmempoolancestors txid (verbose)\nIf txid is in the mempool, returns all in-mempool ancestors."},
        {"blockchain", "getmempooldescendants", getmempooldescendants, true, {"txid", "verbose"}, "getmempooldescendants txid (verbose)\nIf txid is in the mempool, returns all in-mempool descendants."},
        {"blockchain", "getmempoolentry", getmempoolentry, true, {"txid"}, "getmempoolentry txid\nReturns mempool data for given transaction."},
        {"blockchain", "getmempoolinfo", getmempoolinfo, true, {}, "getmempoolinfo\nReturns details on the active state of the TX memory pool."},
        {"blockchain", "getrawmempool", getrawmempool, true, {"verbose"}, "getrawmempool ( verbose )\nReturns all transaction ids in memory pool."},
        {"blockchain", "gettxout", gettxout, true, {"txid", "n", "include_mempool"}, "gettxout \"txid\" n ( include_mempool )\nReturns details about an unspent transaction output."},
        {"blockchain", "gettxoutsetinfo", gettxoutsetinfo, true, {}, "gettxoutsetinfo\nReturns statistics about the unspent transaction output set."},
        {"blockchain", "pruneblockchain", pruneblockchain, true, {"height"}, "pruneblockchain height\nPrune the blockchain up to the given height or timestamp."},
        {"blockchain", "verifychain", verifychain, true, {"checklevel", "nblocks"}, "verifychain ( checklevel nblocks )\nVerifies blockchain database."},
        {"blockchain", "preciousblock", preciousblock, true, {"blockhash"}, "preciousblock \"blockhash\"\nTreats a block as if it were received before others with the same work."},
        {"hidden", "invalidateblock", invalidateblock, true, {"blockhash"}, "invalidateblock \"blockhash\"\nPermanently marks a block as invalid."},
        {"hidden", "reconsiderblock", reconsiderblock, true, {"blockhash"}, "reconsiderblock \"blockhash\"\nRemoves invalidity status of a block and its descendants."},
        {"hidden", "waitfornewblock", waitfornewblock, true, {"timeout"}, "waitfornewblock (timeout)\nWaits for a specific new block and returns useful info about it."},
        {"hidden", "waitforblock", waitforblock, true, {"blockhash", "timeout"}, "waitforblock <blockhash> (timeout)\nWaits for a specific new block."},
        {"hidden", "waitforblockheight", waitforblockheight, true, {"height", "timeout"}, "waitforblockheight <height> (timeout)\nWaits for (at least) block height."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
