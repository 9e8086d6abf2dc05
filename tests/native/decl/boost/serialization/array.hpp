// Declaration-only stand-in (see serialization.hpp).
#pragma once
#include "serialization.hpp"
