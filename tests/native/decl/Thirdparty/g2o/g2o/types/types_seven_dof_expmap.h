// Declaration-only stand-in for the g2o types the reference's Converter.h
// names (its vendored g2o needs Eigen and a generated config.h), for the
// syntax check of adapters/orbslam3/ORBmatcher_searches.cc
// (tests/test_adapter.py).  Test infrastructure; it stands in for no part of
// the reference itself.
#pragma once
namespace g2o {
class SE3Quat;
class Sim3;
}  // namespace g2o
