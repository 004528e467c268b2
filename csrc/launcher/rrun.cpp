// kungfu-rrun: run kungfu-run on every host of -H over ssh (static or elastic).
// Parity: srcs/go/cmd/kungfu-rrun/rrun.go:14-43, srcs/go/utils/runner/remote/remote.go:22-131.
#include "launcher.hpp"

#include <cstdio>

using namespace kungfu;
using namespace kungfu::launcher;

int main(int argc, char **argv) {
    Flags f;
    auto err = f.parse(argc, argv);
    if (!err.empty()) {
        std::fprintf(stderr, "%s\n%s", err.c_str(), Flags::usage().c_str());
        return 2;
    }
    // Forward every flag except -u; each host gets its own -self.
    std::vector<std::string> fwd;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == f.prog) break;
        if (a == "-u") { ++i; continue; }
        fwd.push_back(a);
    }
    HostList hl = f.hosts;
    int rc = 0;
    std::vector<Proc> ps;
    for (auto &h : hl) {
        std::vector<std::string> cmd = {"kungfu-run", "-self", format_ipv4(h.ipv4)};
        cmd.insert(cmd.end(), fwd.begin(), fwd.end());
        cmd.push_back(f.prog);
        cmd.insert(cmd.end(), f.args.begin(), f.args.end());
        Proc p;
        p.name = h.public_addr;
        p.prog = "ssh";
        std::string remote;
        for (auto &c : cmd) remote += (remote.empty() ? "" : " ") + shell_quote(c);
        p.args = {"-o", "StrictHostKeyChecking=no", f.user.empty() ? h.public_addr : f.user + "@" + h.public_addr,
                  remote};
        ps.push_back(p);
    }
    rc = run_all(ps, true, nullptr) ? 1 : 0;
    return rc;
}
