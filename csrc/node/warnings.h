// Node warning state and safe mode (reference src/warnings.{h,cpp}:13-90,
// src/validation.cpp:1203-1297 CheckForkWarningConditions*, src/rpc/server.cpp ObserveSafeMode).
//
// One process-wide warning board, written by the chainstate (unknown block versions, large-work
// forks, a large-work invalid chain) and read by getinfo/getblockchaininfo/getmininginfo/
// getnetworkinfo and by the RPC dispatcher: while any "rpc" warning is up, commands not marked
// okSafeMode fail with RPC_FORBIDDEN_BY_SAFE_MODE unless -disablesafemode is set.
// -testsafemode raises a synthetic warning so the behaviour can be exercised.
#pragma once
#include <string>

namespace bcp {

void SetMiscWarning(const std::string& warning);
std::string GetMiscWarning();
void SetLargeWorkForkFound(bool on);
bool GetLargeWorkForkFound();
void SetLargeWorkInvalidChainFound(bool on);
bool GetLargeWorkInvalidChainFound();

// "statusbar" (everything, newest priority wins), "rpc" (what safe mode keys on) or "gui".
std::string GetWarnings(const std::string& strFor);

// Throws RPC_FORBIDDEN_BY_SAFE_MODE when safe mode is active (see header comment).
void ObserveSafeMode();

} // namespace bcp
