// kungfu-distribute: run an arbitrary command on every host of -H over ssh.
// Parity: srcs/go/cmd/kungfu-distribute/kungfu-distribute.go:22-88.
#include "launcher.hpp"

#include <cstdio>
#include <string>

using namespace kungfu;
using namespace kungfu::launcher;

int main(int argc, char **argv) {
    std::string hosts = "127.0.0.1:1", user;
    int i = 1;
    for (; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-H" && i + 1 < argc) hosts = argv[++i];
        else if (a == "-u" && i + 1 < argc) user = argv[++i];
        else if (a == "--") { ++i; break; }
        else break;
    }
    if (i >= argc) {
        std::fprintf(stderr, "usage: kungfu-distribute -H ip:slots,... [-u user] cmd [args...]\n");
        return 2;
    }
    std::vector<std::string> cmd(argv + i, argv + argc);
    return ssh_run_all(HostList::parse(hosts), user, cmd, true);
}
