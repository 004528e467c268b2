// Local process runner + simple/watch modes + ssh remote launch.
// See launcher.hpp for the parity map.
#include "launcher.hpp"

#include <kungfu/http.hpp>
#include <kungfu/log.hpp>
#include <kungfu/transport.hpp>

#include <fcntl.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <memory>
#include <set>
#include <thread>

extern char **environ;

namespace kungfu {
namespace launcher {

namespace {

const char *kColors[] = {"\033[1;32m", "\033[1;33m", "\033[1;34m", "\033[1;35m", "\033[1;36m", "\033[1;31m"};
std::mutex g_out_mu;

std::atomic<bool> *g_trap_flag = nullptr;

void on_signal(int sig) {
    if (g_trap_flag) g_trap_flag->store(true);
}

void mkdirs(const std::string &dir) {
    std::string cur;
    for (size_t i = 0; i < dir.size(); ++i) {
        cur.push_back(dir[i]);
        if (dir[i] == '/' || i + 1 == dir.size()) ::mkdir(cur.c_str(), 0755);
    }
}

// Streams one fd line by line with a prefix into `out` and optionally a file.
void pump(int fd, FILE *out, const std::string &prefix, const std::string &file, std::string *first_line) {
    std::unique_ptr<std::ofstream> f;
    std::string buf;
    char tmp[8192];
    bool got_first = false;
    auto emit = [&](const std::string &line) {
        if (!got_first && first_line) {
            *first_line = line;
            got_first = true;
        }
        if (!file.empty()) {
            if (!f) f.reset(new std::ofstream(file, std::ios::app));
            *f << line << "\n";
            f->flush();
        }
        if (out) {
            std::lock_guard<std::mutex> lk(g_out_mu);
            std::fprintf(out, "%s%s\n", prefix.c_str(), line.c_str());
            std::fflush(out);
        }
    };
    for (;;) {
        ssize_t n = ::read(fd, tmp, sizeof(tmp));
        if (n <= 0) break;
        buf.append(tmp, static_cast<size_t>(n));
        size_t pos;
        while ((pos = buf.find('\n')) != std::string::npos) {
            emit(buf.substr(0, pos));
            buf.erase(0, pos + 1);
        }
    }
    if (!buf.empty()) emit(buf);
    ::close(fd);
}

int run_once(const Proc &p, int color, bool verbose, const std::string &log_prefix, std::atomic<bool> *cancel,
             std::string *first_stderr) {
    int out_pipe[2], err_pipe[2];
    // O_CLOEXEC: workers forked later must not inherit these write ends, or
    // this worker's output pumps would not see EOF until every sibling exits.
    if (::pipe2(out_pipe, O_CLOEXEC) != 0 || ::pipe2(err_pipe, O_CLOEXEC) != 0) return 127;
    const pid_t parent = ::getpid();
    pid_t pid = ::fork();
    if (pid < 0) return 127;
    if (pid == 0) {
        ::setpgid(0, 0);
        // a worker never outlives its runner (the forking thread waits for it): if the
        // launcher is SIGKILLed (an outer timeout), its GPU workers go with it
        ::prctl(PR_SET_PDEATHSIG, SIGKILL);
        if (::getppid() != parent) ::_exit(127);
        ::dup2(out_pipe[1], 1);
        ::dup2(err_pipe[1], 2);
        ::close(out_pipe[0]);
        ::close(out_pipe[1]);
        ::close(err_pipe[0]);
        ::close(err_pipe[1]);
        for (auto &kv : p.envs) ::setenv(kv.first.c_str(), kv.second.c_str(), 1);
        std::vector<char *> argv;
        argv.push_back(const_cast<char *>(p.prog.c_str()));
        for (auto &a : p.args) argv.push_back(const_cast<char *>(a.c_str()));
        argv.push_back(nullptr);
        ::execvp(p.prog.c_str(), argv.data());
        std::fprintf(stderr, "exec %s failed: %s\n", p.prog.c_str(), std::strerror(errno));
        ::_exit(127);
    }
    ::setpgid(pid, pid);
    ::close(out_pipe[1]);
    ::close(err_pipe[1]);
    bool tty = ::isatty(1);
    std::string c = tty ? kColors[color % 6] : "", r = tty ? "\033[0m" : "";
    std::string pre_out = verbose ? "[" + c + p.name + r + "::stdout] " : "";
    std::string pre_err = verbose ? "[" + c + p.name + r + "::stderr] " : "";
    std::string fout, ferr;
    if (!log_prefix.empty() && !p.logdir.empty()) {
        mkdirs(p.logdir);
        fout = p.logdir + "/" + log_prefix + ".stdout.log";
        ferr = p.logdir + "/" + log_prefix + ".stderr.log";
    }
    std::thread t1(pump, out_pipe[0], verbose ? stdout : nullptr, pre_out, fout, nullptr);
    std::thread t2(pump, err_pipe[0], verbose ? stderr : nullptr, pre_err, ferr, first_stderr);
    int status = 0;
    bool killed = false;
    auto kill_t0 = std::chrono::steady_clock::now();
    for (;;) {
        pid_t w = ::waitpid(pid, &status, WNOHANG);
        if (w == pid) break;
        if (cancel && cancel->load()) {
            if (!killed) {
                ::killpg(pid, SIGTERM);
                killed = true;
                kill_t0 = std::chrono::steady_clock::now();
            } else if (std::chrono::steady_clock::now() - kill_t0 > std::chrono::seconds(5)) {
                ::killpg(pid, SIGKILL);
            }
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    t1.join();
    t2.join();
    if (WIFEXITED(status)) return WEXITSTATUS(status);
    if (WIFSIGNALED(status)) return 128 + WTERMSIG(status);
    return 1;
}

}  // namespace

void trap_signals(std::atomic<bool> *flag) {
    g_trap_flag = flag;
    struct sigaction sa {};
    sa.sa_handler = on_signal;
    sigemptyset(&sa.sa_mask);
    ::sigaction(SIGINT, &sa, nullptr);
    ::sigaction(SIGTERM, &sa, nullptr);
}

int run_proc(const Proc &p, int color, bool verbose, const std::string &log_prefix, std::atomic<bool> *cancel) {
    std::string retry_prefix = env_str("KUNGFU_CONFIG_RETRY_STDERR_PREFIX", "");
    for (int attempt = 1;; ++attempt) {
        std::string first;
        int rc = run_once(p, color, verbose, log_prefix, cancel, &first);
        if (rc != 0 && !retry_prefix.empty() && first.rfind(retry_prefix, 0) == 0 && !(cancel && cancel->load()) &&
            attempt < 10) {
            KF_ERROR("restarting %s for the %d-th time (first stderr line matched retry prefix)", p.name.c_str(),
                     attempt);
            continue;
        }
        return rc;
    }
}

int run_all(const std::vector<Proc> &ps, bool verbose, std::atomic<bool> *cancel) {
    std::atomic<int> fail{0};
    std::atomic<bool> local_cancel{false};
    std::vector<std::thread> ts;
    std::atomic<bool> done{false};
    // propagate the outer cancel flag
    std::thread watcher([&] {
        while (!done.load()) {
            if (cancel && cancel->load()) local_cancel.store(true);
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
    });
    for (size_t i = 0; i < ps.size(); ++i) {
        ts.emplace_back([&, i] {
            std::string prefix = ps[i].name;
            for (auto &c : prefix)
                if (c == '/') c = '-';
            int rc = run_proc(ps[i], static_cast<int>(i), verbose, prefix, &local_cancel);
            if (rc != 0) {
                KF_ERROR("#<%s> exited with error: %d", ps[i].name.c_str(), rc);
                fail++;
                local_cancel.store(true);
            }
        });
    }
    for (auto &t : ts) t.join();
    done.store(true);
    watcher.join();
    return fail.load();
}

int simple_run(uint32_t self_ipv4, const Cluster &cluster, const Job &job, bool verbose, std::atomic<bool> *cancel) {
    auto procs = job.create_procs(cluster, self_ipv4);
    KF_INFO("will parallel run %zu instances of %s", procs.size(), job.prog.c_str());
    auto t0 = std::chrono::steady_clock::now();
    int fails = run_all(procs, verbose, cancel);
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    KF_INFO("all %zu/%zu local peers finished, took %.3fs", procs.size(), cluster.workers.size(), dt);
    if (fails) {
        KF_ERROR("%d tasks failed", fails);
        return 1;
    }
    return 0;
}

// ---- watch mode --------------------------------------------------------------------

namespace {

struct Watcher {
    PeerID self;
    Job job;
    bool keep;
    std::atomic<bool> *cancel;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Stage> stages;
    std::map<int, Stage> versions;
    int running = 0;
    int failures = 0;
    Cluster current;
    std::unique_ptr<GPUPool> pool;
    std::map<uint64_t, std::thread> procs;
    std::set<uint64_t> finished;
    int color = 0;
};

}  // namespace

int watch_run(const PeerID &self, const PeerList &runners, const Stage *init, const Job &job, bool keep,
              int debug_port, std::atomic<bool> *cancel) {
    Watcher w;
    w.self = self;
    w.job = job;
    w.keep = keep;
    w.cancel = cancel;
    w.pool.reset(new GPUPool(std::max(1, job.hosts.slot_of(self.ipv4))));

    Router router(self, env_bool("KUNGFU_CONFIG_USE_UNIX_SOCK", true));
    router.control().set_handler("update", [&](const PeerID &src, const std::string &payload) {
        Stage s;
        try {
            s = Stage::decode(payload);
        } catch (const std::exception &e) {
            KF_WARN("invalid update message: %s", e.what());
            return;
        }
        std::lock_guard<std::mutex> lk(w.mu);
        auto it = w.versions.find(s.version);
        if (it != w.versions.end()) {
            if (!(it->second.cluster == s.cluster)) fatalf("inconsistent update detected at v%d", s.version);
            return;
        }
        w.versions[s.version] = s;
        w.stages.push_back(s);
        w.cv.notify_all();
    });
    router.control().set_handler("exit", [&](const PeerID &, const std::string &) {
        KF_INFO("exit control message received");
        cancel->store(true);
        w.cv.notify_all();
    });
    Server server(self, &router, env_bool("KUNGFU_CONFIG_USE_UNIX_SOCK", true));
    server.start();
    std::unique_ptr<HttpServer> debug;
    if (debug_port > 0) {
        debug.reset(new HttpServer(static_cast<uint16_t>(debug_port), [&](const HttpRequest &) {
            HttpResponse r;
            r.content_type = "application/json";
            auto v = json::Value::object();
            std::lock_guard<std::mutex> lk(w.mu);
            for (auto &kv : w.versions) v.set(std::to_string(kv.first), json::parse(kv.second.encode()));
            r.body = json::dump(v);
            return r;
        }));
        debug->start();
        KF_INFO("debug server: http://127.0.0.1:%d/", debug_port);
    }
    if (init) {
        std::lock_guard<std::mutex> lk(w.mu);
        w.versions[init->version] = *init;
        w.stages.push_back(*init);
    } else KF_INFO("waiting to be initialized");
    KF_INFO("watching config server");

    auto create = [&](const PeerID &id, const Stage &s) {
        int gpu = w.pool->get();
        if (gpu < 0) KF_ERROR("no free GPU slot for %s", id.str().c_str());
        Proc p = w.job.new_proc(id, gpu, s.version, s.cluster);
        w.running++;
        int color = w.color++;
        w.procs[id.hash()] = std::thread([&, p, gpu, color, id, s] {
            std::string prefix = p.name + "@" + std::to_string(s.version);
            int rc = run_proc(p, color, true, prefix, cancel);
            w.pool->put(gpu);
            std::lock_guard<std::mutex> lk(w.mu);
            if (rc != 0) {
                KF_INFO("%s finished with error: %d", p.name.c_str(), rc);
                w.failures++;
                cancel->store(true);
            }
            w.running--;
            w.finished.insert(id.hash());
            w.cv.notify_all();
        });
    };

    std::unique_lock<std::mutex> lk(w.mu);
    for (;;) {
        w.cv.wait_for(lk, std::chrono::milliseconds(100));
        while (!w.stages.empty()) {
            Stage s = w.stages.front();
            w.stages.pop_front();
            server.set_token(static_cast<uint32_t>(s.version));
            if (!w.current.workers.empty() && w.current.workers.disjoint(s.cluster.workers))
                KF_ERROR("full update detected: %s -> %s", w.current.debug_string().c_str(),
                         s.cluster.debug_string().c_str());
            PeerList del = w.current.workers.minus(s.cluster.workers).on(self.ipv4);
            PeerList add = s.cluster.workers.minus(w.current.workers).on(self.ipv4);
            KF_INFO("arrived at v%d, new np=%zu, local: +%zu/-%zu", s.version, s.cluster.workers.size(), add.size(),
                    del.size());
            for (auto &id : del) {
                auto it = w.procs.find(id.hash());
                if (it == w.procs.end()) continue;
                std::thread t = std::move(it->second);
                w.procs.erase(it);
                lk.unlock();
                t.join();
                lk.lock();
            }
            for (auto &id : add) create(id, s);
            w.current = s.cluster;
        }
        // reap finished threads
        for (auto h : w.finished) {
            auto it = w.procs.find(h);
            if (it != w.procs.end()) {
                std::thread t = std::move(it->second);
                w.procs.erase(it);
                lk.unlock();
                t.join();
                lk.lock();
            }
        }
        w.finished.clear();
        if (cancel->load()) {
            KF_ERROR("canceled");
            break;
        }
        if (w.running == 0 && !w.keep && !w.current.workers.empty() && w.stages.empty()) break;
    }
    std::vector<std::thread> rest;
    for (auto &kv : w.procs) rest.push_back(std::move(kv.second));
    w.procs.clear();
    int failures = w.failures;
    lk.unlock();
    for (auto &t : rest) t.join();
    server.stop();
    if (debug) debug->stop();
    KF_INFO("stop watching");
    return failures ? 1 : 0;
}

// ---- ssh ---------------------------------------------------------------------------------

std::string shell_quote(const std::string &s) {
    std::string out = "'";
    for (char c : s) {
        if (c == '\'') out += "'\\''";
        else out.push_back(c);
    }
    return out + "'";
}

int ssh_run_all(const HostList &hosts, const std::string &user, const std::vector<std::string> &cmd, bool verbose) {
    std::vector<Proc> ps;
    for (auto &h : hosts) {
        Proc p;
        p.name = h.public_addr;
        p.prog = "ssh";
        std::string target = user.empty() ? h.public_addr : user + "@" + h.public_addr;
        std::string remote;
        for (auto &c : cmd) remote += (remote.empty() ? "" : " ") + shell_quote(c);
        p.args = {"-o", "StrictHostKeyChecking=no", target, remote};
        ps.push_back(p);
    }
    return run_all(ps, verbose, nullptr) ? 1 : 0;
}

}  // namespace launcher
}  // namespace kungfu
