// Node startup/shutdown sequence (bcpd).
// Parity: reference src/init.cpp AppInitBasicSetup/ParameterInteraction/AppInitMain
// (12 steps: args + config, datadir lock, logging, chain params, caches, script
// threads, RPC warmup server, chainstate load (LoadBlockIndex/InitBlockIndex/
// RewindBlockIndex/VerifyDB), mempool.dat, wallet, connman start, ZMQ), Shutdown(),
// HelpMessage(), and src/bitcoind.cpp (daemon mode, signal handling, wait loop).
#pragma once
#include <string>

namespace bcp {

std::string HelpMessage();
// Full bcpd lifecycle; returns the process exit code.
int AppMain(int argc, char* argv[]);

} // namespace bcp
