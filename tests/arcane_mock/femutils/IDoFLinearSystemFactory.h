// -*- C++ -*-
// TEST MOCK of femutils/IDoFLinearSystemFactory.h:34-44 (tests/arcane_mock/arcane_mock.hpp).
#ifndef AFEM_MOCK_IDOFLINEARSYSTEMFACTORY_H
#define AFEM_MOCK_IDOFLINEARSYSTEMFACTORY_H

#include "arcane_mock.hpp"

namespace Arcane::FemUtils
{
class DoFLinearSystemImpl;
class IDoFLinearSystemFactory
{
 public:

  virtual ~IDoFLinearSystemFactory() = default;
  virtual DoFLinearSystemImpl* createInstance(ISubDomain* sd, IItemFamily* dof_family, const String& solver_name) = 0;
};
} // namespace Arcane::FemUtils

#endif
