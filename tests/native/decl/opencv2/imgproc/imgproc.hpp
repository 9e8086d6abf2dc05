// Declaration-only stand-in (test infrastructure, tests/test_adapter.py): see
// ../opencv.hpp.
#pragma once
#include "../opencv.hpp"
