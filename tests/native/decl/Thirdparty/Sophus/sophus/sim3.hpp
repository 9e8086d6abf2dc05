// Declaration-only stand-in (see ../../../sophus/sim3.hpp).
#pragma once
#include "../../../sophus/sim3.hpp"
