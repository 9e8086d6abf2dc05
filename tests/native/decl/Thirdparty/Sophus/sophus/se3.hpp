// Declaration-only stand-in (see ../../../sophus/se3.hpp).
#pragma once
#include "../../../sophus/se3.hpp"
