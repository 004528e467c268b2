// Job -> per-worker process specs (env contract).  See launcher.hpp for parity.
#include "launcher.hpp"

#include <kungfu/log.hpp>

#include <unistd.h>

#include <algorithm>
#include <ctime>

namespace kungfu {
namespace launcher {

Proc Job::new_proc(const PeerID &peer, int gpu_id, int init_version, const Cluster &cluster) const {
    Proc p;
    p.name = format_ipv4(peer.ipv4) + "." + std::to_string(peer.port);
    p.prog = prog;
    p.args = args;
    p.logdir = logdir;
    auto &e = p.envs;
    e[kEnvJobStartTimestamp] = std::to_string(start_time);
    e[kEnvProcStartTimestamp] = std::to_string(static_cast<long>(std::time(nullptr)));
    e[kEnvSelfSpec] = peer.str();
    e[kEnvInitRunners] = cluster.runners.str();
    e[kEnvParentID] = parent.str();
    e[kEnvInitPeers] = cluster.workers.str();
    e[kEnvInitClusterVersion] = std::to_string(init_version);
    e[kEnvStrategy] = strategy_name(strategy);
    if (!config_server.empty()) e[kEnvConfigServer] = config_server;
    e["KUNGFU_ALLOW_XGMI"] = allow_xgmi ? "true" : "false";
    int idx = gpu_index(gpu_id);
    e["KUNGFU_HIP_VISIBLE_DEVICES"] = std::to_string(idx);
    // ordinal of the slot among the devices this worker sees (all of the
    // launcher's visible GPUs unless -isolate-gpus): what hipSetDevice takes
    e["KUNGFU_HIP_DEVICE_ORDINAL"] = std::to_string(allow_xgmi ? gpu_id : 0);
    if (!allow_xgmi) {
        // One GPU per worker.  HIP honours HIP_VISIBLE_DEVICES; the CUDA name is
        // kept for frameworks that read it.
        e["HIP_VISIBLE_DEVICES"] = std::to_string(idx);
        e["CUDA_VISIBLE_DEVICES"] = std::to_string(idx);
    }
    if (!std::getenv("PYTHONUNBUFFERED")) e["PYTHONUNBUFFERED"] = "1";
    // Several workers per host each defaulting to one OpenMP thread per CPU oversubscribe
    // the host (CPU training steps measured 35x slower); share the CPUs among the host's
    // slots unless the user chose (torchrun does the same with 1 thread).
    if (!std::getenv("OMP_NUM_THREADS")) {
        int slots = 1;
        for (auto &h : hosts)
            if (h.ipv4 == peer.ipv4) slots = std::max(1, h.slots);
        const long ncpu = ::sysconf(_SC_NPROCESSORS_ONLN);
        e["OMP_NUM_THREADS"] = std::to_string(std::max(1L, (ncpu > 0 ? ncpu : 1) / slots));
    }
    // Keep dmabuf IPC (required for RCCL / HIP IPC on this platform).
    if (!std::getenv("HSA_ENABLE_IPC_MODE_LEGACY")) e["HSA_ENABLE_IPC_MODE_LEGACY"] = "0";
    for (auto &h : hosts)
        if (h.ipv4 == peer.ipv4) p.hostname = h.public_addr;
    return p;
}

std::vector<Proc> Job::create_procs(const Cluster &cluster, uint32_t host) const {
    std::vector<Proc> ps;
    for (auto &self : cluster.workers.on(host)) {
        int local_rank = cluster.workers.local_rank(self);
        ps.push_back(new_proc(self, local_rank, 0, cluster));
    }
    return ps;
}

}  // namespace launcher
}  // namespace kungfu
