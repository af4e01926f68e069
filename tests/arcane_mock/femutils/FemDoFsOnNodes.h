// -*- C++ -*-
// TEST MOCK of femutils/FemDoFsOnNodes.h (tests/arcane_mock/arcane_mock.hpp): NB_DOF DoFs per
// node, DoF local id = node local id * NB_DOF + i (the numbering of FemDoFsOnNodes.cc:71-109 on one
// subdomain whose DoF family was created node by node).
#ifndef AFEM_MOCK_FEMDOFSONNODES_H
#define AFEM_MOCK_FEMDOFSONNODES_H

#include "arcane_mock.hpp"

namespace Arcane
{
class IndexedNodeDoFConnectivityView
{
 public:

  explicit IndexedNodeDoFConnectivityView(Int32 nb_dof)
  : m_k(nb_dof)
  {}
  DoFLocalId dofId(NodeLocalId n, Int32 i) const { return DoFLocalId(n.localId() * m_k + i); }

 private:

  Int32 m_k;
};
} // namespace Arcane

namespace Arcane::FemUtils
{
class FemDoFsOnNodes
{
 public:

  explicit FemDoFsOnNodes(Int32 nb_dof)
  : m_k(nb_dof)
  {}
  IndexedNodeDoFConnectivityView nodeDoFConnectivityView() const { return IndexedNodeDoFConnectivityView(m_k); }

 private:

  Int32 m_k;
};
} // namespace Arcane::FemUtils

#endif
