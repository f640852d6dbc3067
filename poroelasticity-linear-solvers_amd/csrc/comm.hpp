// comm.hpp -- communicators of the distributed solve (one process per GPU).
//
// What the Krylov path needs across ranks:
//   * global sums of a few doubles per iteration (CGS dots, norms, Gram
//     partials): done as an allgather of the per-rank partials followed by a
//     rank-ordered sum on every rank, so every rank gets the bitwise same value
//     and the solve is reproducible run to run (a ring all-reduce is not);
//   * a halo exchange of boundary vector entries before each SpMV
//     (point-to-point, neighbours only under the banded ordering);
//   * setup-time exchange of index lists.
// Backends: CommSelf (one rank), CommRCCL (ncclAllGather / grouped
// ncclSend+ncclRecv over xGMI, on the solver stream), CommCallback
// (host-staged through a caller-supplied allgather, e.g. torch.distributed
// gloo -- lets several ranks share one GPU in tests).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/pls.h"  // pls_allgather_fn

namespace pls {

struct Comm {
    int rank = 0, size = 1;
    virtual ~Comm() = default;
    // d_recv[r * count + j] = rank r's d_send[j]
    virtual void allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) = 0;
    // point-to-point: to peer p send scnt[p] doubles from d_send + soff[p];
    // from peer p receive rcnt[p] doubles into d_recv + roff[p]
    virtual void exchange_dev(const double *d_send, const std::vector<int64_t> &scnt,
                              const std::vector<int64_t> &soff, double *d_recv, const std::vector<int64_t> &rcnt,
                              const std::vector<int64_t> &roff, hipStream_t st) = 0;
    // host allgather of equal-size byte blocks (setup only)
    virtual void allgather_host(const void *send, int64_t bytes, void *recv) = 0;

    // in place: d_vals[j] = sum over ranks (rank order) of d_vals[j]
    void global_sum_dev(double *d_vals, int count, hipStream_t st);
    // alltoallv of int64 lists (setup): out[p] = what peer p sent to me
    void alltoallv_i64(const std::vector<std::vector<int64_t>> &to, std::vector<std::vector<int64_t>> &from);

  private:
    double *scratch_ = nullptr;
    size_t scratch_n_ = 0;
};

struct CommSelf : Comm {
    void allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) override;
    void exchange_dev(const double *, const std::vector<int64_t> &, const std::vector<int64_t> &, double *,
                      const std::vector<int64_t> &, const std::vector<int64_t> &, hipStream_t) override {}
    void allgather_host(const void *send, int64_t bytes, void *recv) override;
};

struct CommCallback : Comm {
    pls_allgather_fn fn = nullptr;
    void *user = nullptr;
    void allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) override;
    void exchange_dev(const double *d_send, const std::vector<int64_t> &scnt, const std::vector<int64_t> &soff,
                      double *d_recv, const std::vector<int64_t> &rcnt, const std::vector<int64_t> &roff,
                      hipStream_t st) override;
    void allgather_host(const void *send, int64_t bytes, void *recv) override;
};

struct CommRCCL : Comm {
    void *nccl = nullptr;  // ncclComm_t
    ~CommRCCL() override;
    void allgather_dev(const double *d_send, int count, double *d_recv, hipStream_t st) override;
    void exchange_dev(const double *d_send, const std::vector<int64_t> &scnt, const std::vector<int64_t> &soff,
                      double *d_recv, const std::vector<int64_t> &rcnt, const std::vector<int64_t> &roff,
                      hipStream_t st) override;
    void allgather_host(const void *send, int64_t bytes, void *recv) override;
};

// 128-byte RCCL unique id
int rccl_unique_id(char out[128]);
CommRCCL *rccl_init(const char id[128], int rank, int size);

}  // namespace pls
