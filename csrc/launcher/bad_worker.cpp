// kungfu-bad-worker: fault injection for the launcher's fail-fast policy.
//   kungfu-bad-worker [-error-after STEPS] [-count N]
// Every worker all-reduces an N-element f32 vector in a loop; rank 0 exits with
// status 1 after STEPS steps, so the other workers block in the next collective
// until kungfu-run cancels them (any failure cancels all, local.go:77-80).
// Parity: tests/go/cmd/kungfu-bad-worker/kungfu-bad-worker.go:14-42.
#include <kungfu/capi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int main(int argc, char **argv) {
    int error_after = 3;
    size_t count = 1 << 16;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string a = argv[i];
        if (a == "-error-after") error_after = std::atoi(argv[i + 1]);
        else if (a == "-count") count = static_cast<size_t>(std::atol(argv[i + 1]));
    }
    if (kungfu_init() != 0) {
        std::fprintf(stderr, "init failed: %s\n", kungfu_last_error());
        return 2;
    }
    const int rank = kungfu_rank(), np = kungfu_size();
    std::vector<float> x(count, 1.0f), y(count, 0.0f);
    for (int step = 0;; ++step) {
        if (rank == 0 && step == error_after) {
            std::fprintf(stderr, "kungfu-bad-worker: rank 0 fails at step %d\n", step);
            std::fflush(stderr);
            std::_Exit(1);
        }
        const std::string name = "bad-worker:" + std::to_string(step);
        if (kungfu_all_reduce(x.data(), y.data(), count, /*f32*/ 10, /*sum*/ 0, name.c_str()) != 0) {
            std::fprintf(stderr, "all-reduce failed: %s\n", kungfu_last_error());
            return 3;
        }
        if (y[0] != static_cast<float>(np)) {
            std::fprintf(stderr, "wrong result %f\n", y[0]);
            return 4;
        }
        std::printf("step %d ok\n", step);
        std::fflush(stdout);
    }
}
