// RCCL over xGMI: ghost-DoF halo exchange and the CG scalar all-reduce.
// One process per GPU; the ncclUniqueId is produced by afem_comm_unique_id on
// rank 0 and broadcast by the caller (torch.distributed in the Python
// driver).  Replaces the reference's IParallelMng traffic: the ghost
// synchronize() of femutils/HypreDoFLinearSystem.cc:299 /
// modules/poisson/FemModule.cc:369 and the PCG dot-product reductions inside
// Hypre (femutils/HypreDoFLinearSystem.cc:731-742).
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "afem_internal.hpp"

namespace afem {

struct Comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // host transport (afem_comm_create_host): the caller's IParallelMng-like
  // callbacks move the halo and the dot-product sums through host memory
  bool host = false;
  bool host_async = false;  // halo_begin hands the exchange to a worker thread, halo_end joins it
  afem_host_transport ht{};
  double* pin = nullptr;  // pinned staging buffer (allreduce / halo)
  size_t pin_n = 0;
  double* stage(size_t n)
  {
    if (n > pin_n) {
      if (pin) (void)hipHostFree(pin);
      pin = nullptr;
      AFEM_HIP(hipHostMalloc(reinterpret_cast<void**>(&pin), n * sizeof(double), hipHostMallocDefault));
      pin_n = n;
    }
    return pin;
  }
};

#define AFEM_NCCL(x)                                                                                  \
  do {                                                                                                \
    ncclResult_t r_ = (x);                                                                            \
    if (r_ != ncclSuccess)                                                                            \
      throw ::afem::Error(AFEM_ERR_COMM, std::string(#x) + " failed: " + ncclGetErrorString(r_));     \
  } while (0)

namespace {
__global__ void k_gather(int64_t n, const int32_t* __restrict__ ids, const double* __restrict__ x,
                         double* __restrict__ out)
{
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = x[ids[t]];
}
__global__ void k_scatter(int64_t n, const int32_t* __restrict__ ids, const double* __restrict__ in,
                          double* __restrict__ x)
{
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) x[ids[t]] = in[t];
}
inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }
}  // namespace

void comm_unique_id(uint8_t* out)
{
  static_assert(sizeof(ncclUniqueId) <= AFEM_UNIQUE_ID_BYTES, "ncclUniqueId larger than the ABI buffer");
  ncclUniqueId id;
  AFEM_NCCL(ncclGetUniqueId(&id));
  memset(out, 0, AFEM_UNIQUE_ID_BYTES);
  memcpy(out, &id, sizeof(id));
}

Comm* comm_create(Ctx& ctx, const uint8_t* idb, int nranks, int rank)
{
  AFEM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, AFEM_ERR_ARG, "afem_comm_create: bad rank/nranks");
  ctx.set_device();
  ncclUniqueId id;
  memcpy(&id, idb, sizeof(id));
  auto* c = new Comm();
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    throw Error(AFEM_ERR_COMM, std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r));
  }
  return c;
}

Comm* comm_create_host(int nranks, int rank, const afem_host_transport* t)
{
  AFEM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, AFEM_ERR_ARG, "afem_comm_create_host: bad rank/nranks");
  AFEM_REQUIRE(t && t->allreduce_sum && t->exchange, AFEM_ERR_ARG, "afem_comm_create_host: missing callbacks");
  auto* c = new Comm();
  c->nranks = nranks;
  c->rank = rank;
  c->host = true;
  c->ht = *t;
  return c;
}

void comm_destroy(Comm* c)
{
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->pin) (void)hipHostFree(c->pin);
  delete c;
}

// AFEM_COMM_SELF=1 (diagnostic): a one-rank communicator runs its collectives
// anyway -- ncclAllReduce over one rank, the halo's ncclSend / ncclRecv to
// itself in one group -- so the RCCL data path (groups, the halo stream and
// its events, the PCG's split exchange) runs on a one-GPU box; a halo may then
// name the own rank as its neighbour (tests/test_gpu_parity.py
// test_rccl_self_loop_*)
bool comm_self_loop()
{
  const char* v = variant("AFEM_COMM_SELF");
  return v && std::atoi(v) == 1;
}

namespace {
bool trivial(const Comm* c) { return !c || (c->nranks == 1 && !comm_self_loop()); }
}  // namespace

void comm_allreduce(Comm* c, Ctx& ctx, double* d, int64_t n)
{
  if (trivial(c) || n <= 0) return;
  if (c->host) {
    double* h = c->stage((size_t)n);
    AFEM_HIP(hipMemcpyAsync(h, d, n * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    AFEM_REQUIRE(c->ht.allreduce_sum(c->ht.user, h, n) == 0, AFEM_ERR_COMM, "host transport: allreduce_sum failed");
    AFEM_HIP(hipMemcpyAsync(d, h, n * sizeof(double), hipMemcpyHostToDevice, ctx.stream));
    ctx.sync();
    return;
  }
  AFEM_NCCL(ncclAllReduce(d, d, (size_t)n, ncclDouble, ncclSum, c->comm, ctx.stream));
}

int comm_nranks(Comm* c) { return c ? c->nranks : 1; }
bool comm_is_host(Comm* c) { return c && c->host; }
void comm_set_host_async(Comm* c, bool on)
{
  AFEM_REQUIRE(c && c->host, AFEM_ERR_ARG, "afem_comm_host_async: not a host-transport communicator");
  c->host_async = on;
}
int comm_rank(Comm* c) { return c ? c->rank : 0; }

void halo_setup(Halo& h, Ctx& ctx, Comm* comm, int n_nbr, const int32_t* nbr, const int64_t* send_cnt,
                const int32_t* send_ids, const int64_t* recv_cnt, const int32_t* recv_ids)
{
  h.comm = comm;
  h.nbr.assign(nbr, nbr + n_nbr);
  h.send_cnt.assign(send_cnt, send_cnt + n_nbr);
  h.recv_cnt.assign(recv_cnt, recv_cnt + n_nbr);
  h.send_off.assign(n_nbr + 1, 0);
  h.recv_off.assign(n_nbr + 1, 0);
  for (int i = 0; i < n_nbr; ++i) {
    h.send_off[i + 1] = h.send_off[i] + send_cnt[i];
    h.recv_off[i + 1] = h.recv_off[i] + recv_cnt[i];
  }
  h.n_send = h.send_off[n_nbr];
  h.n_recv = h.recv_off[n_nbr];
  h.send_ids.alloc(h.n_send);
  h.recv_ids.alloc(h.n_recv);
  h.send_buf.alloc(h.n_send);
  h.recv_buf.alloc(h.n_recv);
  if (h.n_send)
    AFEM_HIP(hipMemcpyAsync(h.send_ids.p, send_ids, h.send_ids.bytes(), hipMemcpyHostToDevice, ctx.stream));
  if (h.n_recv)
    AFEM_HIP(hipMemcpyAsync(h.recv_ids.p, recv_ids, h.recv_ids.bytes(), hipMemcpyHostToDevice, ctx.stream));
  ctx.sync();
}

namespace {
// the RCCL send/recv of the packed buffers on `st`; the group is always
// closed, even after a failed send/recv: an open group would swallow every
// later collective on the communicator (the CG all-reduces) and hang; the
// first error is reported after ncclGroupEnd
void post_sendrecv(Halo& h, hipStream_t st)
{
  AFEM_NCCL(ncclGroupStart());
  ncclResult_t first = ncclSuccess;
  const char* what = "";
  for (size_t i = 0; i < h.nbr.size() && first == ncclSuccess; ++i) {
    if (h.send_cnt[i]) {
      first = ncclSend(h.send_buf.p + h.send_off[i], (size_t)h.send_cnt[i], ncclDouble, h.nbr[i], h.comm->comm, st);
      what = "ncclSend";
    }
    if (first == ncclSuccess && h.recv_cnt[i]) {
      first = ncclRecv(h.recv_buf.p + h.recv_off[i], (size_t)h.recv_cnt[i], ncclDouble, h.nbr[i], h.comm->comm, st);
      what = "ncclRecv";
    }
  }
  const ncclResult_t end = ncclGroupEnd();
  if (first != ncclSuccess)
    throw Error(AFEM_ERR_COMM, std::string("halo exchange: ") + what + " failed: " + ncclGetErrorString(first));
  if (end != ncclSuccess) throw Error(AFEM_ERR_COMM, std::string("ncclGroupEnd failed: ") + ncclGetErrorString(end));
}
}  // namespace

namespace {
// host transport, asynchronous: pack on the context stream, copy the send part
// to the halo's pinned buffer, and let a worker thread wait for that copy and
// run the caller's exchange callback while the context stream computes.  The
// callback thus runs on this worker thread, not the caller's: the transport
// must allow that (afem_comm_host_async's contract in arcanefem_amd.h:
// MPI_THREAD_SERIALIZED or better, a Python callback free to take the GIL)
void host_begin_async(Halo& h, Ctx& ctx, double* x)
{
  Comm* c = h.comm;
  const size_t need = (size_t)(h.n_send + h.n_recv);
  if (need > h.hpin_n) {
    if (h.hpin) (void)hipHostFree(h.hpin);
    h.hpin = nullptr;
    AFEM_HIP(hipHostMalloc(reinterpret_cast<void**>(&h.hpin), need * sizeof(double), hipHostMallocDefault));
    h.hpin_n = need;
  }
  if (!h.ev_packed) AFEM_HIP(hipEventCreateWithFlags(&h.ev_packed, hipEventDisableTiming));
  if (h.n_send) {
    hipLaunchKernelGGL(k_gather, dim3(grid_for(h.n_send, 256)), dim3(256), 0, ctx.stream, h.n_send, h.send_ids.p, x,
                       h.send_buf.p);
    AFEM_LAUNCHED();
    AFEM_HIP(hipMemcpyAsync(h.hpin, h.send_buf.p, h.n_send * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  }
  AFEM_HIP(hipEventRecord(h.ev_packed, ctx.stream));
  AFEM_REQUIRE(!h.worker.joinable(), AFEM_ERR_STATE, "halo_begin: an exchange is already in flight");
  const int dev = ctx.device;
  h.worker_rc = 0;
  h.worker = std::thread([&h, c, dev]() {
    if (hipSetDevice(dev) != hipSuccess || hipEventSynchronize(h.ev_packed) != hipSuccess) {
      h.worker_rc = -1;
      return;
    }
    std::vector<int32_t> nb(h.nbr.begin(), h.nbr.end());
    h.worker_rc = c->ht.exchange(c->ht.user, (int)nb.size(), nb.data(), h.hpin, h.send_cnt.data(), h.hpin + h.n_send,
                                 h.recv_cnt.data());
  });
}

void host_end_async(Halo& h, Ctx& ctx, double* x)
{
  if (!h.worker.joinable()) return;
  h.worker.join();
  AFEM_REQUIRE(h.worker_rc == 0, AFEM_ERR_COMM,
               h.worker_rc < 0 ? "host transport: waiting for the packed halo failed" : "host transport: exchange failed");
  if (h.n_recv) {
    AFEM_HIP(hipMemcpyAsync(h.recv_buf.p, h.hpin + h.n_send, h.n_recv * sizeof(double), hipMemcpyHostToDevice,
                            ctx.stream));
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(h.n_recv, 256)), dim3(256), 0, ctx.stream, h.n_recv, h.recv_ids.p,
                       h.recv_buf.p, x);
    AFEM_LAUNCHED();
  }
}
}  // namespace

void halo_begin(Halo& h, Ctx& ctx, double* x)
{
  if (trivial(h.comm) || h.nbr.empty()) return;
  if (h.comm->host) {
    if (h.comm->host_async)
      host_begin_async(h, ctx, x);
    else
      halo_exchange(h, ctx, x);  // synchronous transport: the whole exchange here
    return;
  }
  if (!h.cs) {
    AFEM_HIP(hipStreamCreateWithFlags(&h.cs, hipStreamNonBlocking));
    AFEM_HIP(hipEventCreateWithFlags(&h.ev_packed, hipEventDisableTiming));
    AFEM_HIP(hipEventCreateWithFlags(&h.ev_done, hipEventDisableTiming));
  }
  if (h.n_send) {
    hipLaunchKernelGGL(k_gather, dim3(grid_for(h.n_send, 256)), dim3(256), 0, ctx.stream, h.n_send, h.send_ids.p, x,
                       h.send_buf.p);
    AFEM_LAUNCHED();
  }
  AFEM_HIP(hipEventRecord(h.ev_packed, ctx.stream));
  AFEM_HIP(hipStreamWaitEvent(h.cs, h.ev_packed, 0));
  post_sendrecv(h, h.cs);
  AFEM_HIP(hipEventRecord(h.ev_done, h.cs));
}

void halo_end(Halo& h, Ctx& ctx, double* x)
{
  if (trivial(h.comm) || h.nbr.empty()) return;
  if (h.comm->host) {
    host_end_async(h, ctx, x);  // no-op unless halo_begin started a worker
    return;
  }
  AFEM_HIP(hipStreamWaitEvent(ctx.stream, h.ev_done, 0));
  if (h.n_recv) {
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(h.n_recv, 256)), dim3(256), 0, ctx.stream, h.n_recv, h.recv_ids.p,
                       h.recv_buf.p, x);
    AFEM_LAUNCHED();
  }
}

void halo_exchange(Halo& h, Ctx& ctx, double* x)
{
  if (trivial(h.comm) || h.nbr.empty()) return;
  if (h.n_send) {
    hipLaunchKernelGGL(k_gather, dim3(grid_for(h.n_send, 256)), dim3(256), 0, ctx.stream, h.n_send, h.send_ids.p, x,
                       h.send_buf.p);
    AFEM_LAUNCHED();
  }
  if (h.comm->host) {
    Comm* c = h.comm;
    double* hb = c->stage((size_t)(h.n_send + h.n_recv));
    if (h.n_send)
      AFEM_HIP(hipMemcpyAsync(hb, h.send_buf.p, h.n_send * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    std::vector<int32_t> nb(h.nbr.begin(), h.nbr.end());
    AFEM_REQUIRE(c->ht.exchange(c->ht.user, (int)nb.size(), nb.data(), hb, h.send_cnt.data(), hb + h.n_send,
                                h.recv_cnt.data()) == 0,
                 AFEM_ERR_COMM, "host transport: exchange failed");
    if (h.n_recv)
      AFEM_HIP(hipMemcpyAsync(h.recv_buf.p, hb + h.n_send, h.n_recv * sizeof(double), hipMemcpyHostToDevice,
                              ctx.stream));
    if (h.n_recv) {
      hipLaunchKernelGGL(k_scatter, dim3(grid_for(h.n_recv, 256)), dim3(256), 0, ctx.stream, h.n_recv, h.recv_ids.p,
                         h.recv_buf.p, x);
      AFEM_LAUNCHED();
    }
    ctx.sync();
    return;
  }
  post_sendrecv(h, ctx.stream);
  if (h.n_recv) {
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(h.n_recv, 256)), dim3(256), 0, ctx.stream, h.n_recv, h.recv_ids.p,
                       h.recv_buf.p, x);
    AFEM_LAUNCHED();
  }
}

}  // namespace afem
