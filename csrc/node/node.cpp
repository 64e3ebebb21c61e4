#include "node/node.h"
#include "node/policy.h"

#include <limits>

namespace bcp {

static NodeContext* g_node = nullptr;
NodeContext* GetNode() { return g_node; }
void SetNode(NodeContext* n) { g_node = n; }

std::unique_ptr<NodeContext> BuildNode(const std::string& chain, const std::string& datadir, bool memoryOnly,
                                       bool wipe, bool useGpu) {
    SelectParams(chain);
    std::unique_ptr<NodeContext> node(new NodeContext());
    node->params = &Params();
    node->datadir = datadir;
    node->useGpu = useGpu;
    fRequireStandard = !gArgs.GetBoolArg("-acceptnonstdtxn", !node->params->RequireStandard());
    node->estimator.reset(new CBlockPolicyEstimator());
    node->mempool.reset(new CTxMemPool(node->estimator.get()));
    ChainstateOptions o;
    o.datadir = datadir;
    o.memoryOnly = memoryOnly;
    o.wipe = wipe;
    o.useGpu = useGpu;
    o.txindex = gArgs.GetBoolArg("-txindex", false);
    o.checkBlockIndex = gArgs.GetBoolArg("-checkblockindex", node->params->DefaultConsistencyChecks());
    o.checkpoints = gArgs.GetBoolArg("-checkpoints", true);
    o.maxBlockSize = (uint64_t)gArgs.GetArg("-excessiveblocksize", (int64_t)DEFAULT_MAX_BLOCK_SIZE);
    o.coinsCacheBytes = (size_t)gArgs.GetArg("-dbcache", (int64_t)450) << 20;
    o.scriptThreads = (int)gArgs.GetArg("-par", (int64_t)0);
    o.maxTipAge = gArgs.GetArg("-maxtipage", DEFAULT_MAX_TIP_AGE);
    o.parallelUtxoMinTx = (size_t)std::max<int64_t>(0, gArgs.GetArg("-parallelutxo", (int64_t)o.parallelUtxoMinTx));
    o.connectInPlace = gArgs.GetBoolArg("-connectinplace", o.connectInPlace);
    o.connectLookahead = gArgs.GetBoolArg("-connectlookahead", o.connectLookahead);
    o.recentBlockBytes = (size_t)std::max<int64_t>(0, gArgs.GetArg("-blockcachemb", (int64_t)(o.recentBlockBytes >> 20))) << 20;
    SetFastPrune(gArgs.GetBoolArg("-fastprune", false) && node->params->NetworkIDString() == "regtest");
    const int64_t prune = gArgs.GetArg("-prune", (int64_t)0);
    // -prune=1: manual pruning only (pruneblockchain RPC), never automatic (reference init.cpp)
    if (prune == 1) o.pruneTarget = std::numeric_limits<uint64_t>::max();
    else if (prune > 1) o.pruneTarget = (uint64_t)prune * 1024 * 1024;
    if (gArgs.IsArgSet("-assumevalid")) o.assumeValid = uint256S(gArgs.GetArg("-assumevalid", ""));
    else o.assumeValid = node->params->GetConsensus().defaultAssumeValid;
    node->chainstate.reset(new Chainstate(*node->params, o));
    node->chainstate->SetMempool(node->mempool.get());
    node->mempool->setSanityCheck(gArgs.GetArg("-checkmempool", node->params->DefaultConsistencyChecks() ? 1 : 0));
    SetChainstate(node->chainstate.get());
    return node;
}

std::unique_ptr<NodeContext> CreateNode(const std::string& chain, const std::string& datadir, bool memoryOnly,
                                        bool useGpu, std::string& err) {
    std::unique_ptr<NodeContext> node = BuildNode(chain, datadir, memoryOnly, false, useGpu);
    if (!node->chainstate->LoadBlockIndex(err) || !node->chainstate->InitBlockIndex(err)) {
        SetChainstate(nullptr);
        return nullptr;
    }
    return node;
}

void ShutdownNode(NodeContext& node) {
    if (node.chainstate) node.chainstate->Shutdown();
    if (GetChainstate() == node.chainstate.get()) SetChainstate(nullptr);
    if (GetNode() == &node) SetNode(nullptr);
}

} // namespace bcp
