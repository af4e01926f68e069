// -*- C++ -*-
// TEST MOCK of femutils/DoFLinearSystem.h (tests/arcane_mock/arcane_mock.hpp):
// the interface the shim implements, restated from femutils/DoFLinearSystem.h:42-110
// (CSRFormatView, DoFLinearSystemImpl), plus the part of DoFLinearSystem
// (:130-260) that BSRFormat::toLinearSystem and the test driver call.
#ifndef AFEM_MOCK_DOFLINEARSYSTEM_H
#define AFEM_MOCK_DOFLINEARSYSTEM_H

#include "arcane_mock.hpp"

namespace Arcane::FemUtils
{
class CSRFormatView
{
 public:

  CSRFormatView() = default;
  CSRFormatView(Span<const Int32> rows, Span<const Int32> matrix_rows_nb_column, Span<const Int32> columns,
                Span<Real> values)
  : m_matrix_rows(rows)
  , m_matrix_rows_nb_column(matrix_rows_nb_column)
  , m_matrix_columns(columns)
  , m_values(values)
  {}
  Span<const Int32> rows() const { return m_matrix_rows; }
  Span<const Int32> rowsNbColumn() const { return m_matrix_rows_nb_column; }
  Span<const Int32> columns() const { return m_matrix_columns; }
  Span<Real> values() { return m_values; }
  Int32 nbRow() { return m_matrix_rows.size(); }
  Int32 nbColumn() { return m_matrix_columns.size(); }
  Int32 nbValue() { return m_values.size(); }

 private:

  Span<const Int32> m_matrix_rows, m_matrix_rows_nb_column, m_matrix_columns;
  Span<Real> m_values;
};

class DoFLinearSystemImpl
{
 public:

  virtual ~DoFLinearSystemImpl() = default;
  virtual void matrixAddValue(DoFLocalId row, DoFLocalId column, Real value) = 0;
  virtual void matrixSetValue(DoFLocalId row, DoFLocalId column, Real value) = 0;
  virtual void eliminateRow(DoFLocalId row, Real value) = 0;
  virtual void eliminateRowColumn(DoFLocalId row, Real value) = 0;
  virtual void solve() = 0;
  virtual VariableDoFReal& solutionVariable() = 0;
  virtual VariableDoFReal& rhsVariable() = 0;
  virtual void setSolverCommandLineArguments(const CommandLineArguments& args) = 0;
  virtual void clearValues() = 0;
  virtual void setCSRValues(const CSRFormatView& csr_view) = 0;
  virtual CSRFormatView& getCSRValues() = 0;
  virtual VariableDoFReal& getForcedValue() = 0;
  virtual VariableDoFBool& getForcedInfo() = 0;
  virtual VariableDoFByte& getEliminationInfo() = 0;
  virtual VariableDoFReal& getEliminationValue() = 0;
  virtual bool hasSetCSRValues() const = 0;
  virtual void setRunner(Runner* r) = 0;
  virtual Runner* runner() const = 0;
};

//! the module-facing wrapper: forwards to the implementation a factory made
class DoFLinearSystem
{
 public:

  explicit DoFLinearSystem(DoFLinearSystemImpl* impl)
  : m_impl(impl)
  {}
  ~DoFLinearSystem() { delete m_impl; }
  void matrixAddValue(DoFLocalId r, DoFLocalId c, Real v) { m_impl->matrixAddValue(r, c, v); }
  void matrixSetValue(DoFLocalId r, DoFLocalId c, Real v) { m_impl->matrixSetValue(r, c, v); }
  void eliminateRow(DoFLocalId r, Real v) { m_impl->eliminateRow(r, v); }
  void eliminateRowColumn(DoFLocalId r, Real v) { m_impl->eliminateRowColumn(r, v); }
  void solve() { m_impl->solve(); }
  void clearValues() { m_impl->clearValues(); }
  void setCSRValues(const CSRFormatView& v) { m_impl->setCSRValues(v); }
  CSRFormatView& getCSRValues() { return m_impl->getCSRValues(); }
  bool hasSetCSRValues() const { return m_impl->hasSetCSRValues(); }
  VariableDoFReal& solutionVariable() { return m_impl->solutionVariable(); }
  VariableDoFReal& rhsVariable() { return m_impl->rhsVariable(); }
  VariableDoFBool& getForcedInfo() { return m_impl->getForcedInfo(); }
  VariableDoFReal& getForcedValue() { return m_impl->getForcedValue(); }
  VariableDoFByte& getEliminationInfo() { return m_impl->getEliminationInfo(); }
  VariableDoFReal& getEliminationValue() { return m_impl->getEliminationValue(); }
  void setRunner(Runner* r) { m_impl->setRunner(r); }

 private:

  DoFLinearSystemImpl* m_impl;
};
} // namespace Arcane::FemUtils

#endif
