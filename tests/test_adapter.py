"""The drop-in adapters.  The ORBextractor adapter (adapters/orbslam3/ORBextractor.cc)
compiles against the reference's own, unmodified include/ORBextractor.h
(include/ORBextractor.h:43-109) and this repository's C ABI.  OpenCV is absent
from the image, so tests/native/cv_decl/ declares the subset of its API that
the header and the adapter use (syntax check only: nothing is linked or run).
Skipped where the reference tree is not present (the GPU box)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF_INC = Path("/root/reference/include")


@pytest.mark.skipif(not (REF_INC / "ORBextractor.h").exists(), reason="reference tree not present")
@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_extractor_adapter_compiles_against_reference_header():
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
           "-I", str(ROOT / "tests" / "native" / "cv_decl"), "-I", str(REF_INC), "-I", str(ROOT / "include"),
           str(ROOT / "adapters" / "orbslam3" / "ORBextractor.cc")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_adapter_uses_only_declared_abi():
    """Every orbx_/orbm_ function the adapters call is declared in include/orb_mi355x.h."""
    import re
    header = (ROOT / "include" / "orb_mi355x.h").read_text()
    declared = set(re.findall(r"\b((?:orbx|orbm|orbs|orbv|orbk)_[a-z0-9_]+)\s*\(", header))
    for src in (ROOT / "adapters" / "orbslam3").glob("*.cc"):
        used = set(re.findall(r"\b((?:orbx|orbm|orbs|orbv|orbk)_[a-z0-9_]+)\s*\(", src.read_text()))
        assert used <= declared, (src.name, used - declared)


# Every Frame / KeyFrame / MapPoint / ORBmatcher member the matcher adapter
# (adapters/orbslam3/ORBmatcher_searches.cc) reads, with the declaration the
# adapter's use assumes, found in the reference's own headers.  The adapter
# itself cannot be compiled here: those headers pull in Eigen, Sophus, g2o
# and boost serialization (Frame.h:25-40, KeyFrame.h:23-39, Converter.h:23-30),
# none of which the image has.
MATCHER_MEMBERS = {
    "Frame.h": [r"float mbf;", r"float mb;", r"int N;", r"std::vector<cv::KeyPoint> mvKeys\b",
                r"std::vector<cv::KeyPoint> mvKeysUn;", r"std::vector<MapPoint\*> mvpMapPoints;",
                r"std::vector<float> mvuRight;", r"DBoW2::FeatureVector mFeatVec;", r"cv::Mat mDescriptors\b",
                r"std::vector<bool> mvbOutlier;", r"static float mfGridElementWidthInv;",
                r"static float mfGridElementHeightInv;", r"vector<float> mvScaleFactors;", r"static float mnMinX;",
                r"static float mnMaxX;", r"static float mnMinY;", r"static float mnMaxY;",
                r"GeometricCamera\* mpCamera\b", r"int Nleft\b", r"inline Sophus::SE3<float> GetPose\(\) const"],
    "KeyFrame.h": [r"const float mfGridElementWidthInv;", r"const float mfGridElementHeightInv;",
                   r"const std::vector<cv::KeyPoint> mvKeysUn;", r"const std::vector<float> mvuRight;",
                   r"const cv::Mat mDescriptors;", r"DBoW2::FeatureVector mFeatVec;",
                   r"const std::vector<float> mvScaleFactors;", r"const int mnMinX;", r"const int mnMinY;",
                   r"const int mnMaxX;", r"const int mnMaxY;", r"std::vector<MapPoint\*> GetMapPointMatches\(\);"],
    "MapPoint.h": [r"float mTrackProjX;", r"float mTrackProjY;", r"float mTrackDepth;", r"float mTrackProjXR;",
                   r"bool mbTrackInView\b", r"int mnTrackScaleLevel\b", r"float mTrackViewCos\b",
                   r"Eigen::Vector3f GetWorldPos\(\);", r"int Observations\(\);", r"bool isBad\(\);",
                   r"cv::Mat GetDescriptor\(\);"],
    "ORBmatcher.h": [r"float mfNNratio;", r"bool mbCheckOrientation;",
                     r"int SearchByProjection\(Frame &F, const std::vector<MapPoint\*> &vpMapPoints, const float th=3, "
                     r"const bool bFarPoints = false, const float thFarPoints = 50.0f\);",
                     r"int SearchByProjection\(Frame &CurrentFrame, const Frame &LastFrame, const float th, "
                     r"const bool bMono\);",
                     r"int SearchByBoW\(KeyFrame \*pKF, Frame &F, std::vector<MapPoint\*> &vpMapPointMatches\);",
                     r"int SearchForInitialization\(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched, "
                     r"std::vector<int> &vnMatches12, int windowSize=10\);"],
    "CameraModels/GeometricCamera.h": [r"virtual Eigen::Vector2f project\(const Eigen::Vector3f & v3D\) = 0;"],
}


@pytest.mark.skipif(not (REF_INC / "Frame.h").exists(), reason="reference tree not present")
def test_matcher_adapter_members_declared_in_reference_headers():
    import re
    for hdr, pats in MATCHER_MEMBERS.items():
        text = (REF_INC / hdr).read_text()
        for pat in pats:
            assert re.search(pat, text), f"{hdr}: no declaration matching {pat!r}"
    # and the adapter reads no member outside that list
    src = (ROOT / "adapters" / "orbslam3" / "ORBmatcher_searches.cc").read_text()
    src = re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", src, flags=re.S))
    used = set(re.findall(r"(?:\.|->)\s*(m[a-z]{0,2}[A-Z]\w*|mbf?|N|Nleft|GetPose|GetMapPointMatches|GetWorldPos|Observations|"
                          r"isBad|GetDescriptor|project)\b", src))
    missing = {u for u in used if not any(re.search(r"\b%s\b" % re.escape(u), p) for ps in MATCHER_MEMBERS.values()
                                          for p in ps)}
    assert not missing, f"adapter members not checked against the reference headers: {missing}"
    assert {"mTrackProjX", "mnTrackScaleLevel", "mvbOutlier", "mFeatVec"} <= used
