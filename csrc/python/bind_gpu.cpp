// Python bindings for the CDNA4 kernels (csrc/kernels/*.hip).
#include "consensus/equihash.h"
#include "kernels/gpu_api.h"
#include "node/gpuverify.h"
#include "python/bind.h"
#include "node/miner.h"
#include "node/sigverify.h"
#include "secp256k1/secp256k1.h"

namespace bcp {
namespace py {

static std::vector<gpu::EhBaseState> states_from(const std::vector<CBlake2b>& sts) {
    std::vector<gpu::EhBaseState> v;
    v.reserve(sts.size());
    for (auto& s : sts) v.push_back(gpu::MakeEhBaseState(s));
    return v;
}

void bind_gpu(pyb::module_& m) {
    m.def("gpu_available", &gpu::GpuAvailable);
    m.def("gpu_device_count", &gpu::DeviceCount);
    m.def("gpu_device_name", &gpu::DeviceName);

    pyb::class_<gpu::EquihashGpuSolver>(m, "EquihashGpuSolver")
        .def(pyb::init<unsigned, unsigned, int, int>(), pyb::arg("n"), pyb::arg("k"), pyb::arg("batch") = 1,
             pyb::arg("device") = -1)
        .def_property_readonly("n", &gpu::EquihashGpuSolver::N)
        .def_property_readonly("k", &gpu::EquihashGpuSolver::K)
        .def_property_readonly("batch", &gpu::EquihashGpuSolver::Batch)
        .def_property_readonly("device_bytes", &gpu::EquihashGpuSolver::DeviceBytes)
        // states: list of EquihashState (header+nonce absorbed) -> per nonce list of minimal solutions
        .def("solve",
             [](gpu::EquihashGpuSolver& s, const std::vector<CBlake2b>& sts) {
                 auto bs = states_from(sts);
                 std::vector<std::vector<std::vector<uint32_t>>> r;
                 {
                     pyb::gil_scoped_release rel;
                     r = s.Solve(bs);
                 }
                 const size_t cbl = s.N() / (s.K() + 1);
                 pyb::list out;
                 for (auto& per : r) {
                     pyb::list l;
                     for (auto& idx : per) l.append(to_bytes(GetMinimalFromIndices(idx, cbl)));
                     out.append(l);
                 }
                 return out;
             })
        .def(
            "launch",
            [](gpu::EquihashGpuSolver& s, const std::vector<CBlake2b>& sts, const gpu::EquihashGpuSolver* after) {
                if (after) s.Launch(states_from(sts), *after);
                else s.Launch(states_from(sts));
            },
            pyb::arg("states"), pyb::arg("after") = nullptr)
        .def("debug_expand_corrupt", [](gpu::EquihashGpuSolver& s, int mode) { return s.DebugExpandCorrupt(mode); })
        .def("collect",
             [](gpu::EquihashGpuSolver& s) {
                 std::vector<std::vector<std::vector<uint32_t>>> r;
                 {
                     pyb::gil_scoped_release rel;
                     r = s.Collect();
                 }
                 const size_t cbl = s.N() / (s.K() + 1);
                 pyb::list out;
                 for (auto& per : r) {
                     pyb::list l;
                     for (auto& idx : per) l.append(to_bytes(GetMinimalFromIndices(idx, cbl)));
                     out.append(l);
                 }
                 return out;
             })
        // Launch+collect many batches back to back; returns total solutions (for benchmarking).
        .def("run_nonces",
             [](gpu::EquihashGpuSolver& s, const std::vector<CBlake2b>& sts) {
                 auto bs = states_from(sts);
                 uint64_t total = 0;
                 pyb::gil_scoped_release rel;
                 const size_t B = s.Batch();
                 for (size_t off = 0; off < bs.size(); off += B) {
                     std::vector<gpu::EhBaseState> chunk(bs.begin() + off, bs.begin() + std::min(bs.size(), off + B));
                     auto r = s.Solve(chunk);
                     for (auto& per : r) total += per.size();
                 }
                 return total;
             })
        .def("stats",
             [](const gpu::EquihashGpuSolver& s) {
                 auto& st = s.Stats();
                 pyb::dict d;
                 d["nonces"] = st.nonces;
                 d["candidates"] = st.candidates;
                 d["duplicates"] = st.duplicates;
                 d["solutions"] = st.solutions;
                 d["dropped_rows_sampled"] = st.dropped_rows;
                 d["cand_dropped"] = st.cand_dropped;
                 d["cand_max"] = st.cand_max;
                 d["gpu_ms"] = st.gpu_ms;
                 d["stage_rows"] = st.stage_rows;
                 d["stage_dropped"] = st.stage_dropped;
                 d["stage_maxfill"] = st.stage_maxfill;
                 d["stage_top"] = st.stage_top;
                 d["pair_dropped"] = st.pair_dropped;
                 d["stage_dropped_all"] = st.stage_dropped_all;
                 d["pair_dropped_all"] = st.pair_dropped_all;
                 d["stage_maxfill_all"] = st.stage_maxfill_all;
                 d["overflow_fills"] = st.overflow_fills;
                 d["debug_cands"] = st.debug_cands;
                 return d;
             })
        .def("reset_stats", &gpu::EquihashGpuSolver::ResetStats)
        .def("set_debug", &gpu::EquihashGpuSolver::SetDebug)
        .def("set_stamp_mode", &gpu::EquihashGpuSolver::SetStampMode)
        .def("debug_dump", &gpu::EquihashGpuSolver::DebugDump)
        .def("phase_cycles", &gpu::EquihashGpuSolver::PhaseCycles);

    // Multi-GPU Equihash search of the built-in miner (EquihashSearchGpu) with an accept-all target:
    // returns the first solution found in nonces nonce0+1 .. nonce0+max_nonces (little-endian
    // 256-bit arithmetic on the 32-byte nonce).
    m.def(
        "eh_search_gpu",
        [](unsigned n, unsigned k, const pyb::bytes& input, const pyb::bytes& nonce0, uint64_t maxNonces,
           const std::vector<int>& devices) {
            const auto in = to_vec(input), n0 = to_vec(nonce0);
            if (n0.size() != 32) throw std::invalid_argument("nonce0 must be 32 bytes");
            uint256 start;
            memcpy(start.begin(), n0.data(), 32);
            EhSearchResult r;
            {
                pyb::gil_scoped_release rel;
                r = EquihashSearchGpu(n, k, in, start, maxNonces,
                                      [](const uint256&, const std::vector<unsigned char>&) { return true; }, devices);
            }
            pyb::dict d;
            d["found"] = r.found;
            d["nonce"] = to_bytes(r.nonce.begin(), 32);
            d["solution"] = to_bytes(r.solution.data(), r.solution.size());
            d["nonces"] = r.nonces;
            d["solutions"] = r.solutions;
            return d;
        },
        pyb::arg("n"), pyb::arg("k"), pyb::arg("input"), pyb::arg("nonce0"), pyb::arg("max_nonces"),
        pyb::arg("devices") = std::vector<int>{});

    m.def(
        "eh_verify_batch_gpu",
        [](unsigned n, unsigned k, const std::vector<CBlake2b>& sts, const std::vector<pyb::bytes>& sols, int device) {
            auto bs = states_from(sts);
            std::vector<std::vector<unsigned char>> v;
            for (auto& b : sols) v.push_back(to_vec(b));
            std::vector<uint8_t> r;
            {
                pyb::gil_scoped_release rel;
                r = gpu::EquihashVerifyBatch(n, k, bs, v, device);
            }
            return std::vector<bool>(r.begin(), r.end());
        },
        pyb::arg("n"), pyb::arg("k"), pyb::arg("states"), pyb::arg("solutions"), pyb::arg("device") = -1);

    m.def(
        "sha256d_batch_gpu",
        [](const std::vector<pyb::bytes>& msgs, int device) {
            std::vector<unsigned char> data;
            std::vector<uint64_t> offs;
            std::vector<uint32_t> lens;
            for (auto& b : msgs) {
                std::string s = b;
                offs.push_back(data.size());
                lens.push_back((uint32_t)s.size());
                data.insert(data.end(), s.begin(), s.end());
            }
            std::vector<unsigned char> out;
            {
                pyb::gil_scoped_release rel;
                out = gpu::Sha256dBatch(data, offs, lens, device);
            }
            pyb::list l;
            for (size_t i = 0; i < msgs.size(); ++i) l.append(to_bytes(out.data() + 32 * i, 32));
            return l;
        },
        pyb::arg("msgs"), pyb::arg("device") = -1);
    m.def(
        "sha256d64_batch_gpu",
        [](const pyb::bytes& data, int device) {
            auto v = to_vec(data);
            std::vector<unsigned char> out;
            {
                pyb::gil_scoped_release rel;
                out = gpu::Sha256d64Batch(v, device);
            }
            return to_bytes(out);
        },
        pyb::arg("data"), pyb::arg("device") = -1);
    m.def(
        "merkle_root_gpu",
        [](const pyb::bytes& leaves, int device) {
            auto v = to_vec(leaves);
            bool mutated = false;
            std::vector<unsigned char> root;
            {
                pyb::gil_scoped_release rel;
                root = gpu::MerkleRoot(v, &mutated, device);
            }
            return pyb::make_tuple(to_bytes(root), mutated);
        },
        pyb::arg("leaves"), pyb::arg("device") = -1);
    // device-resident entry points: device pointers and a stream handle (torch tensors' data_ptr()
    // and torch.cuda.current_stream().cuda_stream); asynchronous on that stream
    m.def(
        "sha256d64_device",
        [](uintptr_t in, uintptr_t out, size_t n, int device, uintptr_t stream) {
            gpu::Sha256d64Device(reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out), n, device, stream);
        },
        pyb::arg("in_ptr"), pyb::arg("out_ptr"), pyb::arg("n"), pyb::arg("device"), pyb::arg("stream"));
    m.def(
        "short_txids_device",
        [](uint64_t k0, uint64_t k1, uintptr_t in, uintptr_t out, size_t n, int device, uintptr_t stream) {
            gpu::ShortTxIdsDevice(k0, k1, reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out), n, device,
                                  stream);
        },
        pyb::arg("k0"), pyb::arg("k1"), pyb::arg("in_ptr"), pyb::arg("out_ptr"), pyb::arg("n"), pyb::arg("device"),
        pyb::arg("stream"));
    m.def("ecdsa_job_bytes", &gpu::EcdsaJobBytes);
    // batches up to n signatures take the fused latency kernel (0: never; tests pin each path)
    m.def("ecdsa_set_fused_max", &gpu::SetEcdsaFusedMax, pyb::arg("n"));
    m.def("ecdsa_fused_max", &gpu::EcdsaFusedMax);
    m.def("ecdsa_set_split_kernel", &gpu::SetEcdsaSplitKernel, pyb::arg("k"));
    m.def("ecdsa_split_kernel", &gpu::EcdsaSplitKernel);
    m.def(
        "ecdsa_verify_device",
        [](uintptr_t msg, uintptr_t sig, uintptr_t pub, uintptr_t jobs, uintptr_t result, size_t n, int device,
           uintptr_t stream) {
            gpu::EcdsaVerifyDevice(reinterpret_cast<const void*>(msg), reinterpret_cast<const void*>(sig),
                                   reinterpret_cast<const void*>(pub), reinterpret_cast<void*>(jobs),
                                   reinterpret_cast<void*>(result), n, device, stream);
        },
        pyb::arg("msg_ptr"), pyb::arg("sig_ptr"), pyb::arg("pub_ptr"), pyb::arg("jobs_ptr"), pyb::arg("result_ptr"),
        pyb::arg("n"), pyb::arg("device"), pyb::arg("stream"));
    m.def(
        "short_txid_batch_gpu",
        [](uint64_t k0, uint64_t k1, const pyb::bytes& txids, int device) {
            auto v = to_vec(txids);
            if (v.size() % 32) throw std::invalid_argument("txids must be 32-byte hashes");
            pyb::gil_scoped_release rel;
            return gpu::ShortTxIdBatch(k0, k1, v.data(), v.size() / 32, device);
        },
        pyb::arg("k0"), pyb::arg("k1"), pyb::arg("txids"), pyb::arg("device") = -1);
    m.def(
        "sha256d_scan_nonces_gpu",
        [](const pyb::bytes& header80, const pyb::bytes& target_le, uint32_t start, uint64_t count, int device) {
            auto h = to_vec(header80), t = to_vec(target_le);
            if (h.size() != 80 || t.size() != 32) throw std::invalid_argument("header80/target sizes");
            pyb::gil_scoped_release rel;
            return gpu::Sha256dScanNonces(h.data(), t.data(), start, count, device);
        },
        pyb::arg("header80"), pyb::arg("target_le"), pyb::arg("start"), pyb::arg("count"), pyb::arg("device") = -1);

    // ECDSA batch verification: items = [(pubkey, der_sig, msg32)], CPUsemantics = CPubKey::Verify.
    m.def(
        "ecdsa_verify_batch",
        [](const std::vector<std::tuple<pyb::bytes, pyb::bytes, pyb::bytes>>& items, bool use_gpu, int threads) {
            std::vector<DeferredSigCheck> checks(items.size());
            for (size_t i = 0; i < items.size(); i++) {
                if (!checks[i].pubkey.assign(to_vec(std::get<0>(items[i]))) ||
                    !checks[i].sig.assign(to_vec(std::get<1>(items[i]))))
                    throw std::invalid_argument("pubkey longer than 65 or signature longer than 72 bytes");
                auto m32 = to_vec(std::get<2>(items[i]));
                if (m32.size() != 32) throw std::invalid_argument("msg32");
                memcpy(checks[i].sighash.begin(), m32.data(), 32);
            }
            std::vector<uint8_t> res(checks.size());
            double ms = 0;
            {
                pyb::gil_scoped_release nogil;
                WorkerPool pool(std::max(1, threads));
                const int64_t t0 = GetTimeMicros();
                if (use_gpu) {
                    std::vector<const DeferredSigCheck*> ptrs;
                    for (auto& c : checks) ptrs.push_back(&c);
                    res = GpuVerifyDeferred(ptrs);
                } else {
                    pool.ParallelFor(checks.size(), [&](size_t i) {
                        const DeferredSigCheck& c = checks[i];
                        res[i] = secp::VerifySignature(c.pubkey.data(), c.pubkey.size(), c.sig.data(), c.sig.size(),
                                                       c.sighash.begin());
                    }, 16);
                }
                ms = (GetTimeMicros() - t0) / 1000.0;
            }
            std::vector<bool> out(res.begin(), res.end());
            return pyb::make_tuple(out, ms);
        },
        pyb::arg("items"), pyb::arg("use_gpu") = true, pyb::arg("threads") = 8);

    // Block-validation entry point (BatchVerifySignatures): cache-less, GPU when the batch
    // reaches the threshold, CPU fallback when the device path throws. Returns all-valid.
    m.def(
        "sig_batch_verify",
        [](const std::vector<std::tuple<pyb::bytes, pyb::bytes, pyb::bytes>>& items, bool use_gpu, int threads) {
            std::vector<DeferredSigCheck> checks(items.size());
            for (size_t i = 0; i < items.size(); i++) {
                if (!checks[i].pubkey.assign(to_vec(std::get<0>(items[i]))) ||
                    !checks[i].sig.assign(to_vec(std::get<1>(items[i]))))
                    throw std::invalid_argument("pubkey longer than 65 or signature longer than 72 bytes");
                auto m32 = to_vec(std::get<2>(items[i]));
                if (m32.size() != 32) throw std::invalid_argument("msg32");
                memcpy(checks[i].sighash.begin(), m32.data(), 32);
            }
            pyb::gil_scoped_release nogil;
            WorkerPool pool(std::max(1, threads));
            return BatchVerifySignatures(checks, &pool, use_gpu, false, false);
        },
        pyb::arg("items"), pyb::arg("use_gpu") = true, pyb::arg("threads") = 4);
    // GPU verification service (node/gpuverify.h): validation devices / lanes and the sharded
    // batch paths the node uses (ConnectBlock's ECDSA batch, HEADERS Equihash batches).
    m.def("gpu_verify_set_devices", [](const std::vector<int>& d) { GpuVerifyService::Instance().SetDevices(d); });
    m.def("gpu_verify_devices", []() { return GpuVerifyService::Instance().Devices(); });
    m.def("gpu_verify_set_min_shard", [](size_t ecdsa, size_t eh) {
        GpuVerifyService::Instance().SetMinShard(ecdsa, eh);
    });
    m.def("gpu_verify_set_min_device_shard", [](size_t ecdsa, size_t eh) {
        GpuVerifyService::Instance().SetMinDeviceShard(ecdsa, eh);
    });
    // the shard plan a batch of n items would get on the current lanes: (lane, lo, hi) per shard
    m.def("gpu_verify_plan", [](size_t n, bool equihash) {
        std::vector<std::tuple<size_t, size_t, size_t>> out;
        for (const VerifyShard& s : GpuVerifyService::Instance().Plan(n, equihash)) out.emplace_back(s.lane, s.lo, s.hi);
        return out;
    }, pyb::arg("n"), pyb::arg("equihash") = false);
    // the pure planner (no GPU): PlanShards(n, lane devices, min per device, min per lane)
    m.def("plan_shards", [](size_t n, const std::vector<int>& laneDevices, size_t minDev, size_t minLane) {
        std::vector<std::tuple<size_t, size_t, size_t>> out;
        for (const VerifyShard& s : PlanShards(n, laneDevices, minDev, minLane)) out.emplace_back(s.lane, s.lo, s.hi);
        return out;
    });
    m.def("gpu_verify_shutdown", []() {
        pyb::gil_scoped_release nogil;
        GpuVerifyService::Instance().Shutdown();
    });
    m.def("gpu_verify_stats", []() {
        pyb::list lanes;
        for (const auto& L : GpuVerifyService::Instance().Stats()) {
            pyb::dict d;
            d["device"] = L.device;
            d["priority"] = L.priority;
            d["batches"] = L.batches;
            d["items"] = L.items;
            d["fill_us"] = L.fillMicros;
            d["device_us"] = L.deviceMicros;
            lanes.append(d);
        }
        pyb::dict out;
        out["lanes"] = lanes;
        out["sharded_batches"] = GpuVerifyService::Instance().ShardedBatches();
        return out;
    });
    // packed inputs (msg32 | sig64 compact low-S | pub33 compressed), as gpu::EcdsaVerifyBatch
    m.def("gpu_verify_ecdsa_packed", [](const pyb::bytes& msg, const pyb::bytes& sig, const pyb::bytes& pub) {
        auto mv = to_vec(msg), sv = to_vec(sig), pv = to_vec(pub);
        const size_t n = mv.size() / 32;
        if (mv.size() != n * 32 || sv.size() != n * 64 || pv.size() != n * 33)
            throw std::invalid_argument("gpu_verify_ecdsa_packed: sizes");
        std::vector<uint8_t> r;
        {
            pyb::gil_scoped_release nogil;
            r = GpuVerifyService::Instance().Ecdsa(mv.data(), sv.data(), pv.data(), n);
        }
        return std::vector<bool>(r.begin(), r.end());
    });
    m.def("gpu_verify_equihash", [](unsigned n, unsigned k, const std::vector<CBlake2b>& sts,
                                    const std::vector<pyb::bytes>& sols) {
        auto bs = states_from(sts);
        std::vector<std::vector<unsigned char>> v;
        for (auto& b : sols) v.push_back(to_vec(b));
        std::vector<const std::vector<unsigned char>*> ptrs;
        for (auto& x : v) ptrs.push_back(&x);
        std::vector<uint8_t> r;
        {
            pyb::gil_scoped_release nogil;
            r = GpuVerifyService::Instance().Equihash(n, k, bs, ptrs);
        }
        return std::vector<bool>(r.begin(), r.end());
    });
    m.def("get_miner_gpu_devices", &GetMinerGpuDevices);
    m.def("set_miner_gpu_devices", &SetMinerGpuDevices);
    m.def("set_gpu_fault_injection", &SetGpuFaultInjection);
    m.def("set_gpu_sig_threshold", &SetGpuSigThreshold);
    m.def("get_gpu_sig_threshold", &GetGpuSigThreshold);
    m.def("reset_gpu_sig_failures", &ResetGpuSigFailures);
    m.def("gpu_sig_path_disabled", &GpuSigPathDisabled);
    m.def("sig_verify_stats", []() {
        const SigVerifyStats s = GetSigVerifyStats();
        pyb::dict d;
        d["gpu_batches"] = s.gpu_batches;
        d["gpu_sigs"] = s.gpu_sigs;
        d["cpu_sigs"] = s.cpu_sigs;
        d["cache_hits"] = s.cache_hits;
        d["multisig_groups"] = s.multisig_groups;
        d["gpu_failures"] = s.gpu_failures;
        return d;
    });
}

} // namespace py
} // namespace bcp
