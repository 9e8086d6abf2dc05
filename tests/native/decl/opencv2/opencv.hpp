// Declaration-only subset of OpenCV 4.x for the syntax check of
// adapters/orbslam3/ORBmatcher_searches.cc against the reference's headers
// (tests/test_adapter.py): the extractor adapter's subset (../../cv_decl) plus
// the names the reference's Frame / KeyFrame / MapPoint headers and DBoW2
// declare against.  Test infrastructure; it stands in for no part of the
// reference itself.
#pragma once
#include "../../cv_decl/opencv2/opencv.hpp"
#include <string>
// standard headers the real opencv2/core.hpp pulls in (cvstd.hpp, cvstd.inl.hpp)
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <utility>

namespace cv {
class FileNode;
class FileNodeIterator;
class FileStorage {
public:
    enum Mode { READ = 0, WRITE = 1, APPEND = 2, MEMORY = 4, FORMAT_AUTO = 0, FORMAT_XML = 8, FORMAT_YAML = 16 };
    FileStorage();
    FileStorage(const std::string& filename, int flags, const std::string& encoding = std::string());
    bool open(const std::string& filename, int flags, const std::string& encoding = std::string());
    bool isOpened() const;
    void release();
    FileNode operator[](const std::string& nodename) const;
    FileNode operator[](const char* nodename) const;
    FileNode root(int streamidx = 0) const;
    FileNode getFirstTopLevelNode() const;
};
class FileNode {
public:
    FileNode();
    FileNode operator[](const std::string& nodename) const;
    FileNode operator[](const char* nodename) const;
    FileNode operator[](int i) const;
    bool empty() const;
    bool isNone() const;
    bool isSeq() const;
    bool isMap() const;
    bool isInt() const;
    bool isReal() const;
    bool isString() const;
    size_t size() const;
    std::string string() const;
    double real() const;
    operator int() const;
    operator float() const;
    operator double() const;
    operator std::string() const;
    FileNodeIterator begin() const;
    FileNodeIterator end() const;
};
class FileNodeIterator {
public:
    FileNode operator*() const;
    FileNodeIterator& operator++();
    bool operator!=(const FileNodeIterator&) const;
    bool operator==(const FileNodeIterator&) const;
};
template <typename T> FileStorage& operator<<(FileStorage& fs, const T& value);
FileStorage& operator<<(FileStorage& fs, const std::string& str);
FileStorage& operator<<(FileStorage& fs, const char* str);
void read(const FileNode& node, int& value, int default_value);
void read(const FileNode& node, float& value, float default_value);
void read(const FileNode& node, double& value, double default_value);
void read(const FileNode& node, std::string& value, const std::string& default_value);
void read(const FileNode& node, Mat& mat, const Mat& default_mat = Mat());
template <typename T> void operator>>(const FileNode& n, T& value);
}  // namespace cv

namespace cv {
enum NormTypes { NORM_INF = 1, NORM_L1 = 2, NORM_L2 = 4, NORM_HAMMING = 6 };
class DMatch {
public:
    DMatch();
    DMatch(int queryIdx, int trainIdx, float distance);
    int queryIdx, trainIdx, imgIdx;
    float distance;
};
class BFMatcher {
public:
    BFMatcher(int normType = NORM_L2, bool crossCheck = false);
    void knnMatch(InputArray queryDescriptors, InputArray trainDescriptors,
                  std::vector<std::vector<DMatch>>& matches, int k) const;
};
}  // namespace cv

namespace cv {
std::ostream& operator<<(std::ostream& out, const Mat& mtx);
}  // namespace cv
