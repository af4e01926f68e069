// test mock (tests/arcane_mock/arcane_mock.hpp): the Arcane header of the same path
#include "arcane_mock.hpp"
