/* C ABI of the kungfu-amd runtime (libkungfu_amd.so).
 *
 * Parity: the reference exports GoKungfu* from its cgo archive and wraps them
 * in kungfu::Peer / libkungfu_python (srcs/go/libkungfu-comm/{main,collective,
 * adapt,monitoring}.go, srcs/cpp/include/kungfu/python/init.h:4-31).  Here the
 * runtime is C++, so the ABI is a thin extern "C" layer over kungfu::Peer.
 *
 * Conventions: functions return 0 on success, non-zero on error (message via
 * kungfu_last_error()).  dtype / op codes follow kungfu::DType / ReduceOp.
 * Async variants take a callback invoked from a runtime thread on completion
 * (errors are reported through the callback's status argument — the
 * reference silently drops async errors, libkungfu-comm/main.go:174).
 */
#ifndef KUNGFU_AMD_CAPI_H
#define KUNGFU_AMD_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*kungfu_callback_t)(int status, void *arg);

int kungfu_init(void);  /* from env (single mode if KUNGFU_SELF_SPEC unset) */
int kungfu_init_explicit(const char *self, const char *peers, const char *strategy, int version);
int kungfu_finalize(void);
const char *kungfu_last_error(void);

uint64_t kungfu_uid(void);
int kungfu_detached(void);
int kungfu_rank(void);
int kungfu_size(void);
int kungfu_local_rank(void);
int kungfu_local_size(void);
int kungfu_host_count(void);
int kungfu_cluster_version(void);

int kungfu_barrier(void);
int kungfu_consensus(const void *data, size_t len, const char *name, int *ok);
int kungfu_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name);
int kungfu_all_reduce_async(const void *send, void *recv, size_t count, int dtype, int op, const char *name,
                            kungfu_callback_t cb, void *arg);
int kungfu_cross_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name);
int kungfu_monitored_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name,
                                const int32_t *tree, int tree_len);
int kungfu_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name);
int kungfu_broadcast(const void *send, void *recv, size_t count, int dtype, const char *name);
int kungfu_local_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name);
int kungfu_local_broadcast(const void *send, void *recv, size_t count, int dtype, const char *name);
int kungfu_gather(const void *send, size_t count, int dtype, void *recv, const char *name);
int kungfu_all_gather(const void *send, size_t count, int dtype, void *recv, const char *name);
/* gather to rank 0 -> rank 0 runs transform(gathered [np x count], out, arg) -> broadcast out_bytes of out */
typedef void (*kungfu_transform_t)(const void *gathered, void *out, void *arg);
int kungfu_all_gather_transform(const void *send, size_t count, int dtype, void *out, size_t out_bytes,
                                kungfu_transform_t transform, void *arg, const char *name);

int kungfu_save(const char *name, const void *data, size_t len);
int kungfu_save_version(const char *version, const char *name, const void *data, size_t len);
int kungfu_request(int rank, const char *version, const char *name, void *buf, size_t len, int *found);

int kungfu_propose_new_size(int n);
int kungfu_resize_cluster(int n, int *changed, int *detached);
int kungfu_resize_cluster_from_url(int *changed, int *detached);
int kungfu_set_tree(const int32_t *tree, int n);
int kungfu_calc_stats(void);
int kungfu_log_stats(void);
int kungfu_check_interference(int *switch_strategy);
int kungfu_get_egress_rates(float *rates, int n);
int kungfu_get_peer_latencies(float *lat, int n);

/* host reduction kernel: z = op(x, y) */
int kungfu_transform2(void *z, const void *x, const void *y, size_t n, int dtype, int op);

#ifdef __cplusplus
}
#endif

#endif /* KUNGFU_AMD_CAPI_H */
