/*
 * rpt_gpu_testing.h — test-only seam, compiled ONLY into the test build of the library
 * (tests/loopback/Makefile: rpt_gpu.hip with -DRPT_TESTING_HOOKS=1 -> tests/loopback/build/
 * librpt_gpu_testing.so). The product librpt_gpu.so is built without RPT_TESTING_HOOKS and does not
 * contain this entry point (tests/test_abi.py checks that it is absent).
 *
 * Why: the multi-GPU CREATE_BF Combine (rpt_bf_allreduce_or) drives RCCL through a table
 * of entry points the library fills from librccl on first use. RCCL allows one rank per device, so on
 * a one-GPU box the W-rank choreography of that merge can only run against a stand-in communicator:
 * the loopback RCCL of tests/loopback/rccl_loopback.cpp (W ranks as host threads of one process on one
 * device; grouped send/recv matched at ncclGroupEnd with device-to-device copies). The test loads that
 * library itself and hands its entry points to the test build here.
 */
#ifndef RPT_GPU_TESTING_H
#define RPT_GPU_TESTING_H

#include "rpt_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rccl.h ncclUniqueId, passed by value to ncclCommInitRank */
typedef struct rpt_rccl_unique_id {
  char internal[RPT_RCCL_UNIQUE_ID_BYTES];
} rpt_rccl_unique_id;

/* The rccl.h entry points rpt_bf_allreduce_or / rpt_rccl_* use (ncclResult_t = int, ncclComm_t = void*,
 * hipStream_t = void*, ncclDataType_t / ncclRedOp_t = int). */
typedef struct rpt_rccl_api_table {
  int (*get_unique_id)(rpt_rccl_unique_id* out);                                  /* ncclGetUniqueId */
  int (*comm_init_rank)(void** comm, int nranks, rpt_rccl_unique_id id, int rank); /* ncclCommInitRank */
  int (*comm_destroy)(void* comm);                                                 /* ncclCommDestroy */
  int (*group_start)(void);                                                        /* ncclGroupStart */
  int (*group_end)(void);                                                          /* ncclGroupEnd */
  int (*send)(const void* buf, size_t count, int dtype, int peer, void* comm, void* stream);  /* ncclSend */
  int (*recv)(void* buf, size_t count, int dtype, int peer, void* comm, void* stream);        /* ncclRecv */
  int (*all_reduce)(const void* sendbuf, void* recvbuf, size_t count, int dtype, int op, void* comm,
                    void* stream);                                                 /* ncclAllReduce */
  int (*comm_count)(void* comm, int* count);                                       /* ncclCommCount */
  int (*comm_user_rank)(void* comm, int* rank);                                    /* ncclCommUserRank */
  const char* (*error_string)(int result);                                         /* ncclGetErrorString */
  int (*comm_abort)(void* comm);                                                   /* ncclCommAbort */
  int (*get_async_error)(void* comm, int* async_error);                            /* ncclCommGetAsyncError */
  int (*comm_init_rank_config)(void** comm, int nranks, rpt_rccl_unique_id id, int rank,
                               void* config);                                      /* ncclCommInitRankConfig */
  int (*comm_finalize)(void* comm);                                                /* ncclCommFinalize */
} rpt_rccl_api_table;

#ifdef RPT_TESTING_HOOKS
/* Test build only: route the library's RCCL calls through `table` (copied) instead of librccl; NULL
 * restores librccl. Communicators made through one table must be used and destroyed through it. */
int rpt_testing_set_rccl_api(const rpt_rccl_api_table* table);
/* Test build only: the row count above which rpt_bf_insert_ws runs a bucketed insert in batches (2^31 in
 * the product, 2^20 here, so the batching runs at test sizes). */
uint64_t rpt_testing_bucketed_insert_batch(void);
/* Test build only: on != 0 makes every later bucketed level 1 hit its chunk bound (the never-expected
 * error path: the probe must then pass every row and the insert set every filter bit). */
void rpt_testing_force_l1_error(int on);
#endif

#ifdef __cplusplus
}
#endif

#endif /* RPT_GPU_TESTING_H */
