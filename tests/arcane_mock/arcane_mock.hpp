// -*- C++ -*-
/*
 * TEST INFRASTRUCTURE -- a minimal, single-subdomain stand-in for the part of
 * the Arcane 3.14 API that the shim (shim/AfemDoFLinearSystem.cc,
 * shim/BSRFormat.h) uses, so the shim can be compiled here and driven on the
 * GPU box (tests/test_gpu_shim.py, tests/shim_driver.cpp).  It is NOT Arcane:
 * items are dense local ids of one subdomain, variables are host arrays,
 * IParallelMng is one rank, RunQueue work is synchronous.  Only the names,
 * argument types and meanings the shim relies on are modelled, after their use
 * in the reference (femutils/HypreDoFLinearSystem.cc, femutils/BSRFormat.h,
 * femutils/FemDoFsOnNodes.cc, modules/poisson/FemModule.cc).  Nothing of it
 * is shipped or linked into libafem.
 */
#ifndef AFEM_ARCANE_MOCK_HPP
#define AFEM_ARCANE_MOCK_HPP

#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace Arcane
{
using Int32 = int32_t;
using Int64 = int64_t;
using Integer = Int32;
using Real = double;
using Byte = unsigned char;

struct Real3
{
  Real x = 0, y = 0, z = 0;
};

class String
{
 public:

  String() = default;
  String(const char* c)
  : m_s(c)
  {}
  String(std::string c)
  : m_s(std::move(c))
  {}
  friend String operator+(const String& a, const char* b) { return String(a.m_s + b); }
  bool operator==(const char* b) const { return m_s == b; }
  const std::string& str() const { return m_s; }
  friend std::ostream& operator<<(std::ostream& o, const String& x) { return o << x.m_s; }

 private:

  std::string m_s;
};

// ------------------------------------------------------------------ views / arrays
template <class T>
class Span
{
 public:

  Span() = default;
  Span(T* p, Int64 n)
  : m_p(p)
  , m_n(n)
  {}
  template <class U>
  Span(const Span<U>& o)
  : m_p(o.data())
  , m_n(o.size())
  {}
  T* data() const { return m_p; }
  Int64 size() const { return m_n; }
  T& operator[](Int64 i) const { return m_p[i]; }
  T* begin() const { return m_p; }
  T* end() const { return m_p + m_n; }

 private:

  T* m_p = nullptr;
  Int64 m_n = 0;
};

template <class T>
class ArrayView
{
 public:

  ArrayView() = default;
  ArrayView(Int32 n, T* p)
  : m_p(p)
  , m_n(n)
  {}
  T* data() const { return m_p; }
  Int32 size() const { return m_n; }
  T& operator[](Int32 i) const { return m_p[i]; }
  T* begin() const { return m_p; }
  T* end() const { return m_p + m_n; }

 private:

  T* m_p = nullptr;
  Int32 m_n = 0;
};

template <class T>
class ConstArrayView
{
 public:

  ConstArrayView() = default;
  ConstArrayView(Int32 n, const T* p)
  : m_p(p)
  , m_n(n)
  {}
  const T* data() const { return m_p; }
  Int32 size() const { return m_n; }
  const T& operator[](Int32 i) const { return m_p[i]; }
  const T* begin() const { return m_p; }
  const T* end() const { return m_p + m_n; }

 private:

  const T* m_p = nullptr;
  Int32 m_n = 0;
};
using Int32ConstArrayView = ConstArrayView<Int32>;

template <class T>
class UniqueArray
{
 public:

  UniqueArray() = default;
  UniqueArray(Int64 n, T v)
  : m_v(n, v)
  {}
  void add(const T& x) { m_v.push_back(x); }
  void resize(Int64 n) { m_v.resize(n); }
  void fill(const T& x) { std::fill(m_v.begin(), m_v.end(), x); }
  T& operator[](Int64 i) { return m_v[i]; }
  const T& operator[](Int64 i) const { return m_v[i]; }
  T* data() { return m_v.data(); }
  Int64 size() const { return (Int64)m_v.size(); }
  ArrayView<T> view() { return ArrayView<T>((Int32)m_v.size(), m_v.data()); }
  operator ArrayView<T>() { return view(); }

 private:

  std::vector<T> m_v;
};

// ------------------------------------------------------------------ traces / errors
class ITraceMng
{};

class TraceMessage
{
 public:

  explicit TraceMessage(bool on)
  : m_on(on)
  {}
  ~TraceMessage()
  {
    if (m_on)
      std::cerr << m_os.str() << "\n";
  }
  template <class T>
  TraceMessage& operator<<(const T& x)
  {
    m_os << x;
    return *this;
  }

 private:

  bool m_on;
  std::ostringstream m_os;
};

class TraceAccessor
{
 public:

  explicit TraceAccessor(ITraceMng* tm)
  : m_tm(tm)
  {}
  TraceMessage info() const { return TraceMessage(std::getenv("AFEM_MOCK_TRACE") != nullptr); }
  ITraceMng* traceMng() const { return m_tm; }

 private:

  ITraceMng* m_tm;
};

class FatalErrorException : public std::runtime_error
{
 public:

  using std::runtime_error::runtime_error;
};
class NotImplementedException : public std::runtime_error
{
 public:

  using std::runtime_error::runtime_error;
};
class ArgumentException : public std::runtime_error
{
 public:

  using std::runtime_error::runtime_error;
};

namespace mock
{
  inline void fmt_args(std::vector<std::string>&) {}
  template <class A, class... R>
  void fmt_args(std::vector<std::string>& out, const A& a, const R&... r)
  {
    std::ostringstream os;
    os << a;
    out.push_back(os.str());
    fmt_args(out, r...);
  }
  //! Arcane's "{0} ... {1}" message formatting
  template <class... A>
  std::string format(const char* f, const A&... a)
  {
    std::vector<std::string> v;
    fmt_args(v, a...);
    std::string s(f);
    for (size_t i = 0; i < v.size(); ++i) {
      const std::string key = "{" + std::to_string(i) + "}";
      for (size_t p = s.find(key); p != std::string::npos; p = s.find(key, p + v[i].size()))
        s.replace(p, key.size(), v[i]);
    }
    return s;
  }
} // namespace mock

#define ARCANE_FATAL(...) throw ::Arcane::FatalErrorException(::Arcane::mock::format(__VA_ARGS__))
#define ARCANE_THROW(EX, ...) throw ::Arcane::EX(::Arcane::mock::format(__VA_ARGS__))
#define ARCANE_CHECK_POINTER(p) \
  do { \
    if (!(p)) \
      throw ::Arcane::ArgumentException("null pointer: " #p); \
  } while (0)

namespace platform
{
  inline Real getRealTime()
  {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
} // namespace platform

// ------------------------------------------------------------------ parallel (one rank)
namespace Parallel
{
  enum eReduceType
  {
    ReduceMin,
    ReduceMax,
    ReduceSum
  };
  class Request
  {};
} // namespace Parallel

//! the ranks of a mock job: threads of one process sharing this world
//! (buffered point-to-point mailboxes, barrier-based collectives)
class MockWorld
{
 public:

  explicit MockWorld(Int32 n)
  : m_n(n)
  , m_red(n)
  {}
  Int32 size() const { return m_n; }
  void barrier()
  {
    std::unique_lock<std::mutex> l(m_mu);
    const long g = m_gen;
    if (++m_arrived == m_n) {
      m_arrived = 0;
      ++m_gen;
      m_cv.notify_all();
    }
    else
      m_cv.wait(l, [&] { return m_gen != g; });
  }
  void post(Int32 src, Int32 dst, std::vector<Real> data)
  {
    std::lock_guard<std::mutex> l(m_mu);
    m_box[{ src, dst }].push_back(std::move(data));
    m_cv.notify_all();
  }
  std::vector<Real> take(Int32 src, Int32 dst)
  {
    std::unique_lock<std::mutex> l(m_mu);
    auto& q = m_box[{ src, dst }];
    m_cv.wait(l, [&] { return !q.empty(); });
    std::vector<Real> v = std::move(q.front());
    q.pop_front();
    return v;
  }
  //! sum over the ranks in rank order (the same bits on every rank)
  void reduceSum(Int32 rank, ArrayView<Real> v)
  {
    m_red[rank].assign(v.begin(), v.end());
    barrier();
    for (Int32 i = 0; i < v.size(); ++i) {
      Real s = 0;
      for (Int32 r = 0; r < m_n; ++r)
        s += m_red[r][i];
      v[i] = s;
    }
    barrier();
  }
  std::vector<Byte> bcast;

 private:

  Int32 m_n;
  std::mutex m_mu;
  std::condition_variable m_cv;
  Int32 m_arrived = 0;
  long m_gen = 0;
  std::map<std::pair<Int32, Int32>, std::deque<std::vector<Real>>> m_box;
  std::vector<std::vector<Real>> m_red;
};

class IParallelMng
{
 public:

  IParallelMng() = default;  // one rank
  IParallelMng(MockWorld* w, Int32 rank)
  : m_w(w)
  , m_rank(rank)
  {}
  Int32 commRank() const { return m_rank; }
  Int32 commSize() const { return m_w ? m_w->size() : 1; }
  bool isParallel() const { return commSize() > 1; }
  void reduce(Parallel::eReduceType t, ArrayView<Real> v)
  {
    if (t != Parallel::ReduceSum)
      throw FatalErrorException("mock: ReduceSum only");
    if (m_w)
      m_w->reduceSum(m_rank, v);
  }
  //! buffered: the data are copied out at once, the request is complete
  Parallel::Request send(ConstArrayView<Real> v, Int32 dst, bool)
  {
    m_w->post(m_rank, dst, std::vector<Real>(v.begin(), v.end()));
    return {};
  }
  //! completed by waitAllRequests
  Parallel::Request recv(ArrayView<Real> v, Int32 src, bool)
  {
    m_pending.emplace_back(v, src);
    return {};
  }
  void waitAllRequests(ArrayView<Parallel::Request>)
  {
    for (auto& [v, src] : m_pending) {
      const std::vector<Real> d = m_w->take(src, m_rank);
      if ((Int32)d.size() != v.size())
        throw FatalErrorException("mock: message size mismatch");
      std::copy(d.begin(), d.end(), v.begin());
    }
    m_pending.clear();
  }
  void broadcast(ArrayView<Byte> v, Int32 root)
  {
    if (!m_w)
      return;
    if (m_rank == root)
      m_w->bcast.assign(v.begin(), v.end());
    m_w->barrier();
    if (m_rank != root)
      std::copy(m_w->bcast.begin(), m_w->bcast.end(), v.begin());
    m_w->barrier();
  }

 private:

  MockWorld* m_w = nullptr;
  Int32 m_rank = 0;
  std::vector<std::pair<ArrayView<Real>, Int32>> m_pending;
};

// ------------------------------------------------------------------ items
template <class Tag>
struct ItemLocalIdT
{
  __host__ __device__ constexpr explicit ItemLocalIdT(Int32 i)
  : m_id(i)
  {}
  __host__ __device__ constexpr Int32 localId() const { return m_id; }
  __host__ __device__ constexpr operator Int32() const { return m_id; }

 private:

  Int32 m_id;
};
struct DoFTag
{};
struct NodeTag
{};
struct CellTag
{};
using DoFLocalId = ItemLocalIdT<DoFTag>;
using NodeLocalId = ItemLocalIdT<NodeTag>;
using CellLocalId = ItemLocalIdT<CellTag>;

class IItemFamily;
class IVariableSynchronizer;

//! an item of a family: local id + ownership (+ the cell's nodes)
class Item
{
 public:

  Item(const IItemFamily* f, Int32 lid)
  : m_f(f)
  , m_lid(lid)
  {}
  Int32 localId() const { return m_lid; }
  bool isOwn() const;
  Int32 nbNode() const;
  Item node(Int32 i) const;

 private:

  const IItemFamily* m_f;
  Int32 m_lid;
};
using DoF = Item;
using Node = Item;
using Cell = Item;

class ItemEnumerator
{
 public:

  // holds the group's ids: ENUMERATE_* over a temporary group (group.own())
  // outlives the temporary
  ItemEnumerator(const IItemFamily* f, std::shared_ptr<const std::vector<Int32>> ids)
  : m_f(f)
  , m_ids(std::move(ids))
  {}
  bool hasNext() const { return m_i < m_ids->size(); }
  void operator++() { ++m_i; }
  Int32 itemLocalId() const { return (*m_ids)[m_i]; }
  Item operator*() const { return Item(m_f, itemLocalId()); }

 private:

  const IItemFamily* m_f;
  std::shared_ptr<const std::vector<Int32>> m_ids;
  size_t m_i = 0;
};

class ItemGroup
{
 public:

  ItemGroup() = default;
  ItemGroup(const IItemFamily* f, std::vector<Int32> ids)
  : m_f(f)
  , m_ids(std::make_shared<std::vector<Int32>>(std::move(ids)))
  {}
  Int32 size() const { return (Int32)m_ids->size(); }
  ItemGroup own() const;
  ItemEnumerator enumerator() const { return ItemEnumerator(m_f, m_ids); }

 private:

  const IItemFamily* m_f = nullptr;
  std::shared_ptr<std::vector<Int32>> m_ids;
};
using DoFGroup = ItemGroup;
using NodeGroup = ItemGroup;
using CellGroup = ItemGroup;

#define AFEM_MOCK_ENUMERATE(name, group) for (auto name = (group).enumerator(); name.hasNext(); ++name)
#define ENUMERATE_DOF(name, group) AFEM_MOCK_ENUMERATE(name, group)
#define ENUMERATE_NODE(name, group) AFEM_MOCK_ENUMERATE(name, group)
#define ENUMERATE_CELL(name, group) AFEM_MOCK_ENUMERATE(name, group)

//! per communicating rank: the owned items it receives from us (shared) and
//! our ghosts it owns (FemDoFsOnNodes::computeSynchronizeInfos' lists)
class IVariableSynchronizer
{
 public:

  Int32ConstArrayView communicatingRanks() const { return Int32ConstArrayView((Int32)ranks.size(), ranks.data()); }
  Int32ConstArrayView sharedItems(Int32 i) const { return Int32ConstArrayView((Int32)shared[i].size(), shared[i].data()); }
  Int32ConstArrayView ghostItems(Int32 i) const { return Int32ConstArrayView((Int32)ghosts[i].size(), ghosts[i].data()); }
  std::vector<Int32> ranks;
  std::vector<std::vector<Int32>> shared, ghosts;
};

//! a family of items with dense local ids 0..n-1; cells carry their nodes
class IItemFamily
{
 public:

  IItemFamily(Int32 n, Int32 n_own, IParallelMng* pm, ITraceMng* tm)
  : m_n(n)
  , m_n_own(n_own)
  , m_pm(pm)
  , m_tm(tm)
  {}
  ITraceMng* traceMng() const { return m_tm; }
  IParallelMng* parallelMng() const { return m_pm; }
  Int32 maxLocalId() const { return m_n; }
  //! the owned items are lids [0, n_own) unless an ownership mask was set
  bool isOwn(Int32 lid) const { return m_own_mask.empty() ? lid < m_n_own : m_own_mask[lid] != 0; }
  void setOwnMask(std::vector<char> m) { m_own_mask = std::move(m); }
  ItemGroup allItems() const
  {
    std::vector<Int32> ids(m_n);
    for (Int32 i = 0; i < m_n; ++i)
      ids[i] = i;
    return ItemGroup(this, std::move(ids));
  }
  ItemGroup ownItems() const
  {
    std::vector<Int32> ids;
    for (Int32 i = 0; i < m_n; ++i)
      if (isOwn(i))
        ids.push_back(i);
    return ItemGroup(this, std::move(ids));
  }
  IVariableSynchronizer* allItemsSynchronizer() { return &m_sync; }
  // cells: nv nodes per item
  std::vector<Int32> cell_node;
  Int32 nv = 0;

 private:

  Int32 m_n, m_n_own;
  IParallelMng* m_pm;
  ITraceMng* m_tm;
  std::vector<char> m_own_mask;
  IVariableSynchronizer m_sync;
};

inline bool Item::isOwn() const { return m_f->isOwn(m_lid); }
inline Int32 Item::nbNode() const { return m_f->nv; }
inline Item Item::node(Int32 i) const { return Item(nullptr, m_f->cell_node[(size_t)m_lid * m_f->nv + i]); }
inline ItemGroup ItemGroup::own() const
{
  std::vector<Int32> ids;
  for (Int32 lid : *m_ids)
    if (m_f->isOwn(lid))
      ids.push_back(lid);
  return ItemGroup(m_f, std::move(ids));
}

// ------------------------------------------------------------------ variables
struct VariableBuildInfo
{
  VariableBuildInfo(IItemFamily* f, const String& name)
  : family(f)
  , name(name)
  {}
  IItemFamily* family;
  String name;
};

template <class LID, class T>
class ItemVariableScalarRefT
{
 public:

  explicit ItemVariableScalarRefT(const VariableBuildInfo& vbi)
  : m_family(vbi.family)
  , m_v(vbi.family->maxLocalId())
  {}
  ItemVariableScalarRefT(Int32 n)
  : m_v(n)
  {}
  void fill(const T& x) { std::fill(m_v.begin(), m_v.end(), x); }
  T& operator[](LID i) { return m_v[i.localId()]; }
  const T& operator[](LID i) const { return m_v[i.localId()]; }
  //! the owners' values into the ghosts (Real variables, over the family's synchronizer)
  void synchronize()
  {
    if constexpr (std::is_same_v<T, Real>) {
      if (!m_family || !m_family->parallelMng()->isParallel())
        return;
      IParallelMng* pm = m_family->parallelMng();
      IVariableSynchronizer* sync = m_family->allItemsSynchronizer();
      const Int32ConstArrayView ranks = sync->communicatingRanks();
      std::vector<std::vector<Real>> in(ranks.size());
      for (Int32 i = 0; i < ranks.size(); ++i) {
        std::vector<Real> out;
        for (Int32 lid : sync->sharedItems(i))
          out.push_back(m_v[lid]);
        pm->send(ConstArrayView<Real>((Int32)out.size(), out.data()), ranks[i], false);
        in[i].resize(sync->ghostItems(i).size());
        pm->recv(ArrayView<Real>((Int32)in[i].size(), in[i].data()), ranks[i], false);
      }
      pm->waitAllRequests({});
      for (Int32 i = 0; i < ranks.size(); ++i) {
        Int32 k = 0;
        for (Int32 lid : sync->ghostItems(i))
          m_v[lid] = in[i][k++];
      }
    }
  }
  Int32 size() const { return (Int32)m_v.size(); }

 private:

  IItemFamily* m_family = nullptr;
  std::deque<T> m_v;  // deque<bool> holds real bools (operator[] returns bool&)
};
using VariableDoFReal = ItemVariableScalarRefT<DoFLocalId, Real>;
using VariableDoFBool = ItemVariableScalarRefT<DoFLocalId, bool>;
using VariableDoFByte = ItemVariableScalarRefT<DoFLocalId, Byte>;
using VariableNodeReal3 = ItemVariableScalarRefT<NodeLocalId, Real3>;

// ------------------------------------------------------------------ mesh
class IMesh
{
 public:

  IMesh(Int32 dim, IItemFamily* nodes, IItemFamily* cells, IParallelMng* pm)
  : m_dim(dim)
  , m_nodes(nodes)
  , m_cells(cells)
  , m_pm(pm)
  , m_coords(nodes->maxLocalId())
  {}
  Int32 dimension() const { return m_dim; }
  IParallelMng* parallelMng() const { return m_pm; }
  IItemFamily* nodeFamily() const { return m_nodes; }
  IItemFamily* cellFamily() const { return m_cells; }
  NodeGroup ownNodes() const { return m_nodes->ownItems(); }
  NodeGroup allNodes() const { return m_nodes->allItems(); }
  CellGroup allCells() const { return m_cells->allItems(); }
  VariableNodeReal3& nodesCoordinates() { return m_coords; }

 private:

  Int32 m_dim;
  IItemFamily *m_nodes, *m_cells;
  IParallelMng* m_pm;
  VariableNodeReal3 m_coords;
};

// ------------------------------------------------------------------ accelerator
enum class eExecutionPolicy
{
  None,
  Sequential,
  Thread,
  HIP
};
enum class eMemoryRessource
{
  Host,
  Device
};
class Runner
{
 public:

  explicit Runner(eExecutionPolicy p)
  : m_p(p)
  {}
  eExecutionPolicy executionPolicy() const { return m_p; }

 private:

  eExecutionPolicy m_p;
};
namespace Accelerator
{
  inline bool isAcceleratorPolicy(eExecutionPolicy p) { return p == eExecutionPolicy::HIP; }
} // namespace Accelerator
class RunQueue
{
 public:

  explicit RunQueue(eMemoryRessource m)
  : m_mem(m)
  {}
  void barrier() { (void)hipDeviceSynchronize(); }
  eMemoryRessource memoryRessource() const { return m_mem; }

 private:

  eMemoryRessource m_mem;
};

struct MDDim1
{};
//! NumArray<Int32, MDDim1> in host or device memory (the queue's resource)
template <class T, class Dim>
class NumArray
{
 public:

  NumArray() = default;
  NumArray(Int64 n, eMemoryRessource m)
  : m_mem(m)
  {
    resize(n);
  }
  NumArray(const NumArray&) = delete;
  NumArray& operator=(NumArray&& o) noexcept
  {
    std::swap(m_p, o.m_p);
    std::swap(m_n, o.m_n);
    std::swap(m_mem, o.m_mem);
    return *this;
  }
  ~NumArray() { release(); }
  void resize(Int64 n)
  {
    release();
    m_n = n;
    if (m_mem == eMemoryRessource::Device)
      (void)hipMalloc(&m_p, sizeof(T) * (n > 0 ? n : 1));
    else
      m_p = static_cast<T*>(std::malloc(sizeof(T) * (n > 0 ? n : 1)));
  }
  void copy(ConstArrayView<T> src)
  {
    (void)hipMemcpy(m_p, src.data(), sizeof(T) * src.size(), hipMemcpyDefault);
  }
  Span<T> to1DSpan() { return Span<T>(m_p, m_n); }

 private:

  void release()
  {
    if (!m_p)
      return;
    if (m_mem == eMemoryRessource::Device)
      (void)hipFree(m_p);
    else
      std::free(m_p);
    m_p = nullptr;
  }
  T* m_p = nullptr;
  Int64 m_n = 0;
  eMemoryRessource m_mem = eMemoryRessource::Host;
};

// ------------------------------------------------------------------ services
class CommandLineArguments
{};
class ISubDomain
{};
struct ServiceBuildInfo
{
  ITraceMng* tm = nullptr;
};

//! name -> factory of the registered services (ARCANE_REGISTER_SERVICE_*)
template <class Base>
std::map<std::string, std::function<Base*(const ServiceBuildInfo&)>>& mockServiceRegistry()
{
  static std::map<std::string, std::function<Base*(const ServiceBuildInfo&)>> r;
  return r;
}

} // namespace Arcane

using namespace Arcane;

#endif
