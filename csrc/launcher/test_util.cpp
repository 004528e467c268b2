// kungfu-test-util: fault injection / control-plane poking for tests.
//   kungfu-test-util -kill ip:port [ip:port ...]       send the "exit" control message
//   kungfu-test-util -control NAME ip:port [payload]   send any control message
// Parity: tests/go/cmd/kungfu-test-util/kungfu-test-util.go:58-65 (kill a peer through
// the control channel, handled by srcs/go/rchannel/handler/control.go:17-23).
#include <kungfu/transport.hpp>

#include <cstdio>
#include <string>
#include <vector>

using namespace kungfu;

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: kungfu-test-util -kill ip:port [...] | -control NAME ip:port [payload]\n");
        return 2;
    }
    std::string mode = argv[1];
    // The client only needs a source identity for the connection header; nothing listens on it.
    Client client(PeerID::parse("127.0.0.1:1"), /*use_uds=*/false);
    try {
        if (mode == "-kill") {
            for (int i = 2; i < argc; ++i) {
                auto dst = PeerID::parse(argv[i]);
                client.send(dst, ConnType::CONTROL, "exit", nullptr, 0);
                std::printf("sent exit to %s\n", dst.str().c_str());
            }
        } else if (mode == "-control" && argc >= 4) {
            std::string payload = argc >= 5 ? argv[4] : "";
            auto dst = PeerID::parse(argv[3]);
            client.send(dst, ConnType::CONTROL, argv[2], payload.data(), payload.size());
            std::printf("sent %s to %s\n", argv[2], dst.str().c_str());
        } else {
            std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
            return 2;
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "kungfu-test-util: %s\n", e.what());
        return 1;
    }
    client.close_all();
    return 0;
}
