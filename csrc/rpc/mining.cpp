// Mining RPCs. Parity: reference src/rpc/mining.cpp (command table :1147):
// getnetworkhashps, getmininginfo, prioritisetransaction, getblocktemplate (BIP22/23
// incl. longpoll and proposal mode), submitblock (optional `legacy` format flag :913-988),
// generate/generatetoaddress (GPU Equihash/SHA256d search), estimatefee/priority(+smart).
#include "consensus/merkle.h"
#include "consensus/pow.h"
#include "keys/key.h"
#include "net/net.h"
#include "node/miner.h"
#include "node/node.h"
#include "node/signals.h"
#include "node/txmempool.h"
#include "rpc/core_io.h"
#include "rpc/server.h"
#include "script/standard.h"
#include "util/strencodings.h"

#include <cmath>

namespace bcp {

static NodeContext& Node() {
    NodeContext* n = GetNode();
    if (!n || !n->chainstate) ThrowRPC(RPC_INTERNAL_ERROR, "node not initialised");
    return *n;
}
double GetDifficulty(const CBlockIndex* blockindex);

static UniValue GetNetworkHashPS(int lookup, int height) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    CBlockIndex* pb = cs.Tip();
    if (height >= 0 && height < cs.Height()) pb = cs.ActiveChain()[height];
    if (pb == nullptr || !pb->nHeight) return 0;
    if (lookup <= 0) lookup = pb->nHeight % cs.Params().GetConsensus().DifficultyAdjustmentInterval() + 1;
    if (lookup > pb->nHeight) lookup = pb->nHeight;
    CBlockIndex* pb0 = pb;
    int64_t minTime = pb0->GetBlockTime(), maxTime = minTime;
    for (int i = 0; i < lookup; i++) {
        pb0 = pb0->pprev;
        const int64_t t = pb0->GetBlockTime();
        minTime = std::min(t, minTime);
        maxTime = std::max(t, maxTime);
    }
    if (minTime == maxTime) return 0;
    const arith_uint256 workDiff = pb->nChainWork - pb0->nChainWork;
    const int64_t timeDiff = maxTime - minTime;
    return workDiff.getdouble() / timeDiff;
}

static UniValue getnetworkhashps(const JSONRPCRequest& req) {
    Chainstate& cs = *Node().chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    return GetNetworkHashPS(req.params.size() > 0 && !req.params[0].isNull() ? req.params[0].get_int() : 120,
                            req.params.size() > 1 && !req.params[1].isNull() ? req.params[1].get_int() : -1);
}

static CScript ScriptForAddress(const std::string& addr, const CChainParams& params) {
    CTxDestination dest = DecodeDestination(addr, params);
    if (!dest.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Error: Invalid address");
    return GetScriptForDestination(dest);
}

static UniValue generateBlocks(const CScript& script, int nGenerate, uint64_t nMaxTries) {
    NodeContext& n = Node();
    std::string err;
    std::vector<uint256> hashes = GenerateBlocks(*n.chainstate, n.mempool.get(), script, nGenerate, nMaxTries, n.useGpu, &err);
    if (!err.empty()) ThrowRPC(RPC_INTERNAL_ERROR, err);
    UniValue blockHashes(UniValue::VARR);
    for (const uint256& h : hashes) blockHashes.push_back(h.GetHex());
    return blockHashes;
}

// Coinbase script for `generate`: the wallet's next key when a wallet is loaded,
// otherwise a fixed node key (reference requires a wallet; see GetScriptForMining).
CScript GetScriptForMining();

static UniValue generate(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "generate nblocks ( maxtries )");
    const int nGenerate = req.params[0].get_int();
    uint64_t nMaxTries = 1000000;
    if (req.params.size() > 1 && !req.params[1].isNull()) nMaxTries = (uint64_t)req.params[1].get_int64();
    return generateBlocks(GetScriptForMining(), nGenerate, nMaxTries);
}

static UniValue generatetoaddress(const JSONRPCRequest& req) {
    if (req.params.size() < 2 || req.params.size() > 3)
        ThrowRPC(RPC_INVALID_PARAMS, "generatetoaddress nblocks address (maxtries)");
    const int nGenerate = req.params[0].get_int();
    uint64_t nMaxTries = 1000000;
    if (req.params.size() > 2 && !req.params[2].isNull()) nMaxTries = (uint64_t)req.params[2].get_int64();
    return generateBlocks(ScriptForAddress(req.params[1].get_str(), Node().chainstate->Params()), nGenerate, nMaxTries);
}

static UniValue getmininginfo(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("blocks", cs.Height());
    obj.pushKV("currentblocksize", (uint64_t)BlockAssembler(cs, n.mempool.get()).LastBlockSize());
    obj.pushKV("currentblocktx", (uint64_t)BlockAssembler(cs, n.mempool.get()).LastBlockTx());
    obj.pushKV("difficulty", GetDifficulty(cs.Tip()));
    obj.pushKV("blockprioritypercentage", (uint8_t)gArgs.GetArg("-blockprioritypercentage", (int64_t)5));
    obj.pushKV("errors", cs.Warnings());
    obj.pushKV("networkhashps", GetNetworkHashPS(120, -1));
    obj.pushKV("pooledtx", (uint64_t)n.mempool->size());
    obj.pushKV("chain", cs.Params().NetworkIDString());
    const MinerStats ms = GetMinerStats();
    UniValue gpu(UniValue::VOBJ);
    gpu.pushKV("enabled", n.useGpu);
    gpu.pushKV("equihash_nonces", (uint64_t)ms.eh_nonces);
    gpu.pushKV("equihash_solutions", (uint64_t)ms.eh_solutions);
    gpu.pushKV("sha256d_nonces", (uint64_t)ms.sha_nonces);
    gpu.pushKV("gpu_ms", ms.gpu_ms);
    obj.pushKV("miner", gpu);
    return obj;
}

static UniValue prioritisetransaction(const JSONRPCRequest& req) {
    if (req.params.size() != 3) ThrowRPC(RPC_INVALID_PARAMS, "prioritisetransaction <txid> <priority delta> <fee delta>");
    const uint256 hash = ParseHashStr(req.params[0].get_str(), "txid");
    const Amount nAmount = req.params[2].get_int64();
    Node().mempool->PrioritiseTransaction(hash, req.params[1].get_real(), nAmount);
    return true;
}

static UniValue BIP22ValidationResult(const CValidationState& state) {
    if (state.IsValid()) return UniValue::NullUniValue;
    const std::string strRejectReason = state.GetRejectReason();
    if (state.IsError()) ThrowRPC(RPC_VERIFY_ERROR, strRejectReason);
    if (state.IsInvalid()) {
        if (strRejectReason.empty()) return "rejected";
        return strRejectReason;
    }
    return "valid?";
}

// BIP9 deployment name as getblocktemplate shows it: '!' marks a rule the client must
// understand (reference src/rpc/mining.cpp:419-426 gbt_vb_name)
static std::string gbt_vb_name(Consensus::DeploymentPos pos) {
    const VBDeploymentInfo& vbinfo = VersionBitsDeploymentInfo[pos];
    std::string s = vbinfo.name;
    if (!vbinfo.gbt_force) s.insert(s.begin(), '!');
    return s;
}

// Parity: reference src/rpc/mining.cpp:428-897 (BIP22/BIP23/BIP9 getblocktemplate), including
// the proposal_legacy mode (an 80-byte-header block), the next-height check of proposals,
// maxversion -> version/force for pre-versionbits clients, and the refusals of a node without
// peers (-9) or in initial block download (-10, regtest included).
static UniValue getblocktemplate(const JSONRPCRequest& req) {
    NodeContext& n = Node();
    Chainstate& cs = *n.chainstate;
    std::string strMode = "template";
    UniValue lpval = UniValue::NullUniValue;
    std::set<std::string> setClientRules;
    int64_t nMaxVersionPreVB = -1;
    if (req.params.size() > 0 && !req.params[0].isNull()) {
        const UniValue& oparam = req.params[0].get_obj();
        const UniValue& modeval = oparam["mode"];
        if (modeval.isStr()) strMode = modeval.get_str();
        else if (!modeval.isNull()) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid mode");
        lpval = oparam["longpollid"];
        if (strMode == "proposal" || strMode == "proposal_legacy") {
            const UniValue& dataval = oparam["data"];
            if (!dataval.isStr()) ThrowRPC(RPC_TYPE_ERROR, "Missing data String key for proposal");
            CBlock block;
            const bool legacy_format = strMode == "proposal_legacy";
            if (!DecodeHexBlk(block, dataval.get_str(), legacy_format))
                ThrowRPC(RPC_DESERIALIZATION_ERROR, "Block decode failed");
            std::lock_guard<CCriticalSection> l(cs.cs());
            const uint256 hash = block.GetHash(cs.Params().GetConsensus());
            CBlockIndex* pindex = cs.LookupBlockIndex(hash);
            if (pindex) {
                if (pindex->IsValid(BLOCK_VALID_SCRIPTS)) return "duplicate";
                if (pindex->nStatus & BLOCK_FAILED_MASK) return "duplicate-invalid";
                return "duplicate-inconclusive";
            }
            CBlockIndex* const pindexPrev = cs.Tip();
            // TestBlockValidity only supports blocks built on the current tip
            if (block.hashPrevBlock != pindexPrev->GetBlockHash()) return "inconclusive-not-best-prevblk";
            // the header's height must be the next one (a legacy-format block carries none, so
            // proposal_legacy always ends here, as in the reference)
            if (block.nHeight != (uint32_t)pindexPrev->nHeight + 1) return "inconclusive-bad-height";
            CValidationState state;
            cs.TestBlockValidity(state, block, pindexPrev, false, true);
            return BIP22ValidationResult(state);
        }
        const UniValue& aClientRules = oparam["rules"];
        if (aClientRules.isArray()) {
            for (size_t i = 0; i < aClientRules.size(); ++i) setClientRules.insert(aClientRules[i].get_str());
        } else {
            // read only from clients that do not speak versionbits
            const UniValue& uvMaxVersion = oparam["maxversion"];
            if (uvMaxVersion.isNum()) nMaxVersionPreVB = uvMaxVersion.get_int64();
        }
    }
    if (strMode != "template") ThrowRPC(RPC_INVALID_PARAMETER, "Invalid mode");
    CConnman* connman = GetConnman();
    if (!connman) ThrowRPC(RPC_CLIENT_P2P_DISABLED, "Error: Peer-to-peer functionality missing or disabled");
    if (connman->GetNodeCount(CONNECTIONS_ALL) == 0) ThrowRPC(RPC_CLIENT_NOT_CONNECTED, "Bitcoin is not connected!");
    if (cs.IsInitialBlockDownload()) ThrowRPC(RPC_CLIENT_IN_INITIAL_DOWNLOAD, "Bitcoin is downloading blocks...");

    static unsigned nTransactionsUpdatedLast;
    if (!lpval.isNull()) {
        // long-poll: wait until the tip or the mempool changed
        uint256 hashWatchedChain;
        unsigned nTransactionsUpdatedLastLP;
        if (lpval.isStr()) {
            const std::string lpstr = lpval.get_str();
            hashWatchedChain.SetHex(lpstr.substr(0, 64));
            nTransactionsUpdatedLastLP = (unsigned)atoi64(lpstr.substr(64));
        } else {
            hashWatchedChain = cs.TipNow()->GetBlockHash();
            nTransactionsUpdatedLastLP = nTransactionsUpdatedLast;
        }
        int64_t checktxtime = GetTimeMillis() + 60000;
        std::unique_lock<CCriticalSection> l(cs.cs());
        AssertLockHeld(cs.cs()); // (unique_lock is invisible to the thread-safety analysis)
        while (cs.Tip()->GetBlockHash() == hashWatchedChain && !ShutdownRequested()) {
            cs.BlockChangeCV().wait_for(l, std::chrono::milliseconds(1000));
            if (GetTimeMillis() > checktxtime) {
                if (n.mempool->GetTransactionsUpdated() != nTransactionsUpdatedLastLP) break;
                checktxtime += 10000;
            }
        }
    }

    static CBlockIndex* pindexPrev = nullptr;
    static int64_t nStart = 0;
    static std::unique_ptr<CBlockTemplate> pblocktemplate;
    static std::mutex csTemplate;
    std::lock_guard<std::mutex> lt(csTemplate);
    std::lock_guard<CCriticalSection> l(cs.cs());
    if (pindexPrev != cs.Tip() ||
        (n.mempool->GetTransactionsUpdated() != nTransactionsUpdatedLast && GetTime() - nStart > 5)) {
        pindexPrev = nullptr;
        nTransactionsUpdatedLast = n.mempool->GetTransactionsUpdated();
        CBlockIndex* pindexPrevNew = cs.Tip();
        nStart = GetTime();
        CScript scriptDummy = CScript() << OP_TRUE;
        pblocktemplate = BlockAssembler(cs, n.mempool.get()).CreateNewBlock(scriptDummy);
        pindexPrev = pindexPrevNew;
    }
    CBlock* pblock = &pblocktemplate->block;
    UpdateTime(pblock, cs.Params().GetConsensus(), pindexPrev);
    pblock->nNonce.SetNull();

    UniValue aCaps(UniValue::VARR);
    aCaps.push_back("proposal");
    UniValue transactions(UniValue::VARR);
    std::map<uint256, int64_t> setTxIndex;
    int i = 0;
    for (const auto& it : pblock->vtx) {
        const CTransaction& tx = *it;
        const uint256 txId = tx.GetHash();
        setTxIndex[txId] = i++;
        if (tx.IsCoinBase()) continue;
        UniValue entry(UniValue::VOBJ);
        entry.pushKV("data", EncodeHexTx(tx));
        entry.pushKV("txid", txId.GetHex());
        entry.pushKV("hash", tx.GetHash().GetHex());
        UniValue deps(UniValue::VARR);
        for (const CTxIn& in : tx.vin)
            if (setTxIndex.count(in.prevout.hash)) deps.push_back(setTxIndex[in.prevout.hash]);
        entry.pushKV("depends", deps);
        const int index_in_template = i - 1;
        entry.pushKV("fee", pblocktemplate->vTxFees[index_in_template]);
        entry.pushKV("sigops", pblocktemplate->vTxSigOpsCount[index_in_template]);
        transactions.push_back(entry);
    }
    UniValue aux(UniValue::VOBJ);
    aux.pushKV("flags", HexStr(std::vector<unsigned char>()));
    arith_uint256 hashTarget = arith_uint256().SetCompact(pblock->nBits);
    UniValue aMutable(UniValue::VARR);
    aMutable.push_back("time");
    aMutable.push_back("transactions");
    aMutable.push_back("prevblock");
    UniValue result(UniValue::VOBJ);
    result.pushKV("capabilities", aCaps);
    UniValue aRules(UniValue::VARR);
    UniValue vbavailable(UniValue::VOBJ);
    for (int j = 0; j < (int)Consensus::MAX_VERSION_BITS_DEPLOYMENTS; ++j) {
        const Consensus::DeploymentPos pos = (Consensus::DeploymentPos)j;
        const ThresholdState state = cs.DeploymentState(pindexPrev, pos);
        const VBDeploymentInfo& vbinfo = VersionBitsDeploymentInfo[pos];
        switch (state) {
        case THRESHOLD_DEFINED:
        case THRESHOLD_FAILED: break;
        case THRESHOLD_LOCKED_IN:
            pblock->nVersion |= VersionBitsMask(cs.Params().GetConsensus(), pos);
            // fallthrough
        case THRESHOLD_STARTED:
            vbavailable.pushKV(gbt_vb_name(pos), cs.Params().GetConsensus().vDeployments[pos].bit);
            if (setClientRules.find(vbinfo.name) == setClientRules.end() && !vbinfo.gbt_force)
                pblock->nVersion &= ~VersionBitsMask(cs.Params().GetConsensus(), pos);
            break;
        case THRESHOLD_ACTIVE:
            aRules.push_back(gbt_vb_name(pos));
            // an active rule the client does not know: only safe when it is gbt_force
            if (setClientRules.find(vbinfo.name) == setClientRules.end() && !vbinfo.gbt_force)
                ThrowRPC(RPC_INVALID_PARAMETER,
                         strprintf("Support for '%s' rule requires explicit client support", vbinfo.name));
            break;
        }
    }
    result.pushKV("version", pblock->nVersion);
    result.pushKV("rules", aRules);
    result.pushKV("vbavailable", vbavailable);
    result.pushKV("vbrequired", 0);
    // a pre-versionbits client (maxversion, no rules) may change the version back to v2: safe
    // only because a non-force active deployment threw above (BIP34 fixed the coinbase layout)
    if (nMaxVersionPreVB >= 2) aMutable.push_back("version/force");
    result.pushKV("previousblockhash", pblock->hashPrevBlock.GetHex());
    result.pushKV("transactions", transactions);
    result.pushKV("coinbaseaux", aux);
    result.pushKV("coinbasevalue", (int64_t)pblock->vtx[0]->vout[0].nValue);
    result.pushKV("longpollid", cs.Tip()->GetBlockHash().GetHex() + std::to_string(nTransactionsUpdatedLast));
    result.pushKV("target", ArithToUint256(hashTarget).GetHex());
    result.pushKV("mintime", (int64_t)pindexPrev->GetMedianTimePast() + 1);
    result.pushKV("mutable", aMutable);
    result.pushKV("noncerange", "00000000ffffffff");
    // the reference reports the default 8 MB limits here, whatever -excessiveblocksize is
    result.pushKV("sigoplimit", (int64_t)GetMaxBlockSigOpsCount(DEFAULT_MAX_BLOCK_SIZE));
    result.pushKV("sizelimit", (int64_t)DEFAULT_MAX_BLOCK_SIZE);
    result.pushKV("curtime", pblock->GetBlockTime());
    result.pushKV("bits", strprintf("%08x", pblock->nBits));
    result.pushKV("height", (int64_t)(pindexPrev->nHeight + 1));
    // BCP: post-fork templates are Equihash work (header nHeight, 256-bit nonce)
    if (cs.IsBCPEnabled(pindexPrev->nHeight + 1))
        result.pushKV("equihash", strprintf("%u,%u", cs.Params().EquihashN(), cs.Params().EquihashK()));
    return result;
}

namespace {
class submitblock_StateCatcher : public CValidationInterface {
public:
    uint256 hash;
    bool found = false;
    CValidationState state;
    const Consensus::Params& cp;
    submitblock_StateCatcher(const uint256& h, const Consensus::Params& p) : hash(h), cp(p) {}
    void BlockChecked(const CBlock& block, const CValidationState& stateIn) override {
        if (block.GetHash(cp) != hash) return;
        found = true;
        state = stateIn;
    }
};
} // namespace

static UniValue submitblock(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 3)
        ThrowRPC(RPC_INVALID_PARAMS, "submitblock \"hexdata\" ( \"jsonparametersobject\" \"legacy\" )");
    Chainstate& cs = *Node().chainstate;
    auto blockptr = std::make_shared<CBlock>();
    const bool legacy = req.params.size() == 3 && req.params[2].get_bool();
    if (!DecodeHexBlk(*blockptr, req.params[0].get_str(), legacy)) ThrowRPC(RPC_DESERIALIZATION_ERROR, "Block decode failed");
    if (blockptr->vtx.empty() || !blockptr->vtx[0]->IsCoinBase())
        ThrowRPC(RPC_DESERIALIZATION_ERROR, "Block does not start with a coinbase");
    const uint256 hash = blockptr->GetHash(cs.Params().GetConsensus());
    bool fBlockPresent = false;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        CBlockIndex* pindex = cs.LookupBlockIndex(hash);
        if (pindex) {
            if (pindex->IsValid(BLOCK_VALID_SCRIPTS)) return "duplicate";
            if (pindex->nStatus & BLOCK_FAILED_MASK) return "duplicate-invalid";
            fBlockPresent = true;
        }
    }
    submitblock_StateCatcher sc(hash, cs.Params().GetConsensus());
    GetMainSignals().Register(&sc);
    CValidationState stateOut;
    const bool fAccepted = cs.ProcessNewBlock(blockptr, true, nullptr, &stateOut);
    GetMainSignals().Unregister(&sc);
    if (fBlockPresent) {
        if (fAccepted && !sc.found) return "duplicate-inconclusive";
        return "duplicate";
    }
    if (!sc.found) {
        // rejected before script checks (e.g. bad PoW/Equihash): report the state directly
        if (!fAccepted && !stateOut.IsValid()) return BIP22ValidationResult(stateOut);
        return "inconclusive";
    }
    return BIP22ValidationResult(sc.state);
}

static UniValue estimatefee(const JSONRPCRequest& req) {
    int nBlocks = req.params[0].get_int();
    if (nBlocks < 1) nBlocks = 1;
    CFeeRate feeRate = Node().mempool->Estimator()->estimateFee(nBlocks);
    if (feeRate == CFeeRate(0)) return -1.0;
    return ValueFromAmount(feeRate.GetFeePerK());
}
static UniValue estimatepriority(const JSONRPCRequest& req) {
    int nBlocks = req.params[0].get_int();
    if (nBlocks < 1) nBlocks = 1;
    return Node().mempool->Estimator()->estimatePriority(nBlocks);
}
static UniValue estimatesmartfee(const JSONRPCRequest& req) {
    const int nBlocks = req.params[0].get_int();
    UniValue result(UniValue::VOBJ);
    int answerFound = 0;
    CFeeRate feeRate = Node().mempool->Estimator()->estimateSmartFee(nBlocks, &answerFound);
    result.pushKV("feerate", feeRate == CFeeRate(0) ? UniValue(-1.0) : ValueFromAmount(feeRate.GetFeePerK()));
    result.pushKV("blocks", answerFound);
    return result;
}
static UniValue estimatesmartpriority(const JSONRPCRequest& req) {
    UniValue result(UniValue::VOBJ);
    int answerFound = 0;
    const double priority = Node().mempool->Estimator()->estimateSmartPriority(req.params[0].get_int(), &answerFound);
    result.pushKV("priority", priority);
    result.pushKV("blocks", answerFound);
    return result;
}

void RegisterMiningRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"mining", "getnetworkhashps", getnetworkhashps, true, {"nblocks", "height"}, "getnetworkhashps ( nblocks height )\nReturns the estimated network hashes per second."},
        {"mining", "getmininginfo", getmininginfo, true, {}, "getmininginfo\nReturns a json object containing mining-related information."},
        {"mining", "prioritisetransaction", prioritisetransaction, true, {"txid", "priority_delta", "fee_delta"}, "prioritisetransaction <txid> <priority delta> <fee delta>\nAccepts the transaction into mined blocks at a higher (or lower) priority."},
        {"mining", "getblocktemplate", getblocktemplate, true, {"template_request"}, "getblocktemplate ( TemplateRequest )\nReturns data needed to construct a block to work on (BIP22/23)."},
        {"mining", "submitblock", submitblock, true, {"hexdata", "parameters", "legacy"}, "submitblock \"hexdata\" ( \"jsonparametersobject\" \"legacy\" )\nAttempts to submit new block to network."},
        {"generating", "generate", generate, true, {"nblocks", "maxtries"}, "generate nblocks ( maxtries )\nMine up to nblocks blocks immediately (GPU Equihash/SHA256d search)."},
        {"generating", "generatetoaddress", generatetoaddress, true, {"nblocks", "address", "maxtries"}, "generatetoaddress nblocks address (maxtries)\nMine blocks immediately to a specified address."},
        {"util", "estimatefee", estimatefee, true, {"nblocks"}, "estimatefee nblocks\nEstimates the approximate fee per kilobyte needed for confirmation within nblocks."},
        {"util", "estimatepriority", estimatepriority, true, {"nblocks"}, "estimatepriority nblocks\nDEPRECATED. Estimates the priority needed for zero-fee confirmation."},
        {"util", "estimatesmartfee", estimatesmartfee, true, {"nblocks"}, "estimatesmartfee nblocks\nEstimates the fee per kilobyte, searching up to higher targets."},
        {"util", "estimatesmartpriority", estimatesmartpriority, true, {"nblocks"}, "estimatesmartpriority nblocks\nDEPRECATED."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
