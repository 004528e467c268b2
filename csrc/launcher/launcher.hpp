// kungfu-run launcher: flags, job/env contract, GPU slot pool, local process
// runner (prefixed/coloured output + per-proc log files, fail-fast), simple and
// watch (elastic) modes.
//
// Parity (reference paths relative to /root/reference/srcs/go):
//   kungfu-run main            cmd/kungfu-run/app/kungfu-run.go:18-112
//   flags                      kungfu/runner/flags.go:29-137
//   builtin config server      cmd/kungfu-run/app/builtin-config-server.go:13-27
//   Job / NewProc env          kungfu/job/job.go:31-98
//   GPU pool / visible devices kungfu/job/gpu_resource.go:11-51, job/cuda_visible_device.go:17-58
//   SimpleRun / RunAll         kungfu/runner/simple.go:13-21, utils/runner/local/local.go:62-92
//   retry on known crash       utils/runner/local/hack.go:14-35 (here: configurable stderr prefix)
//   watch mode + handler       kungfu/runner/watch.go:23-150, kungfu/runner/handler.go:19-123
//   InferSelfIPv4              kungfu/runner/discovery.go:18-60
//   xterm/log redirect         utils/iostream/{xterm,lazyfile}.go
//   remote launch              utils/runner/remote/remote.go, cmd/kungfu-rrun, cmd/kungfu-distribute
//
// ROCm specifics: the per-worker GPU slot is exported as KUNGFU_HIP_VISIBLE_DEVICES.
// By default every GPU stays visible to every worker and the worker selects its
// slot (hipSetDevice): RCCL's intra-node P2P/IPC transport over xGMI needs the
// peers' devices to be visible, otherwise it falls back to a host-memory path.
// -isolate-gpus (or -allow-xgmi=false) restores the reference's default of one
// visible GPU per worker (HIP_VISIBLE_DEVICES=<slot>, job/job.go:31-98).
#pragma once

#include <kungfu/peer.hpp>
#include <kungfu/plan.hpp>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace kungfu {
namespace launcher {

struct Flags {
    int np = 1;
    std::string host_list_str;
    std::string hostfile;
    HostList hosts;
    std::string user;
    PortRange port_range;
    std::string self;
    double timeout = 0;
    bool verbose = true;
    std::string nic;
    bool allow_xgmi = true;
    Strategy strategy = Strategy::BINARY_TREE_STAR;
    int port = kDefaultRunnerPort;
    int debug_port = 0;
    bool watch = false;
    bool keep = false;
    int init_version = 0;
    std::string config_server;
    long job_start_time = 0;
    std::string logfile;
    std::string logdir;
    bool quiet = false;
    double delay = 0;
    int builtin_config_port = 0;
    std::string platform;  // "" or "modelarts"
    std::string prog;
    std::vector<std::string> args;

    // Parses argv (Go-flag style: -name value, -name=value, bool -name).
    // Returns "" on success, an error message otherwise.
    std::string parse(int argc, char **argv);
    static std::string usage();
};

uint32_t infer_self_ipv4(const std::string &self, const std::string &nic);
// ... and, with neither hint, the local IPv4 that appears in the host list
uint32_t infer_self_ipv4(const std::string &self, const std::string &nic, const HostList &hosts);
std::vector<uint32_t> local_ipv4s();

// Platform peer discovery (ModelArts DLS_* / BATCH_CUSTOM<i>_HOSTS env).
struct ContainerInfo {
    PeerID self;
    PeerList runners;
};
ContainerInfo parse_modelarts_env();

// GPU id of a local rank given the visible-devices env (HIP/ROCR/CUDA).
int gpu_index(int local_rank);
std::vector<int> parse_visible_devices(const std::string &val, bool *ok);

class GPUPool {
  public:
    explicit GPUPool(int n) : mask_(n, true) {}
    int get();
    void put(int id);

  private:
    std::mutex mu_;
    std::vector<bool> mask_;
};

struct Proc {
    std::string name;
    std::string prog;
    std::vector<std::string> args;
    std::map<std::string, std::string> envs;
    std::string hostname;
    std::string logdir;
};

struct Job {
    long start_time = 0;
    std::string config_server;
    Strategy strategy = Strategy::BINARY_TREE_STAR;
    PeerID parent;
    HostList hosts;
    PortRange port_range;
    std::string prog;
    std::vector<std::string> args;
    std::string logdir;
    bool allow_xgmi = true;

    Proc new_proc(const PeerID &peer, int gpu_id, int init_version, const Cluster &cluster) const;
    std::vector<Proc> create_procs(const Cluster &cluster, uint32_t host) const;
};

// Runs one process to completion, streaming output.  Returns exit status
// (0 ok).  `cancel` (if set) kills the process group.  Retries when the first
// stderr line starts with KUNGFU_CONFIG_RETRY_STDERR_PREFIX.
int run_proc(const Proc &p, int color, bool verbose, const std::string &log_prefix, std::atomic<bool> *cancel);

// Fail-fast parallel run: any failure cancels the rest.  Returns #failures.
int run_all(const std::vector<Proc> &ps, bool verbose, std::atomic<bool> *cancel);

int simple_run(uint32_t self_ipv4, const Cluster &cluster, const Job &job, bool verbose, std::atomic<bool> *cancel);
int watch_run(const PeerID &self, const PeerList &runners, const Stage *init, const Job &job, bool keep,
              int debug_port, std::atomic<bool> *cancel);

// Installs SIGINT/SIGTERM handlers that set *flag.
void trap_signals(std::atomic<bool> *flag);

// Remote launch over ssh.
int ssh_run_all(const HostList &hosts, const std::string &user, const std::vector<std::string> &cmd, bool verbose);
std::string shell_quote(const std::string &s);

int kungfu_run_main(int argc, char **argv);

}  // namespace launcher
}  // namespace kungfu
