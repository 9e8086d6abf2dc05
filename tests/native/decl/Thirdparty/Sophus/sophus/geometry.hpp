// Declaration-only stand-in (see ../../../sophus/geometry.hpp).
#pragma once
#include "../../../sophus/geometry.hpp"
