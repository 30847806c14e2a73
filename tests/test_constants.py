"""Known-answer pins read from the reference text (tests/golden/constants_fixture.json, made by
tests/golden/make_pattern_fixture.py): the constants of ORBextractor.cc:71-73 and
ORBmatcher.cc:37-39 as the oracle and the HIP library use them, and the ORB parameters of
Examples/ORB_RGB640x480.yaml:35-48 as the bench uses them.  CPU only: the library getter needs
no device."""
import json
import os

import bench
import oracle
from orbslam_mapsave_amd import native

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "constants_fixture.json")


def _fixture():
    with open(GOLDEN) as f:
        return json.load(f)


def test_fixture_cites_reference_lines():
    fx = _fixture()
    assert set(fx["constants"]) == set(oracle.CONSTANT_NAMES)
    for name, e in fx["constants"].items():
        src = e["source"]
        assert src.startswith("src/ORBextractor.cc:" if name in
                              ("PATCH_SIZE", "HALF_PATCH_SIZE", "EDGE_THRESHOLD")
                              else "src/ORBmatcher.cc:")


def test_oracle_constants_match_reference():
    fx = _fixture()["constants"]
    assert oracle.reference_constants() == {k: v["value"] for k, v in fx.items()}


def test_hip_library_constants_match_reference():
    fx = _fixture()["constants"]
    assert native.reference_constants() == {k: v["value"] for k, v in fx.items()}


def test_bench_parameters_match_yaml():
    y = {k: v["value"] for k, v in _fixture()["yaml_ORB_RGB640x480"].items()}
    assert (bench.ORB_SCALE, bench.ORB_LEVELS, bench.ORB_INI_TH, bench.ORB_MIN_TH) == (
        y["scaleFactor"], y["nLevels"], y["iniThFAST"], y["minThFAST"])
    assert bench.ORB_YAML_NFEATURES == y["nFeatures"]
    # the oracle's tables for those parameters: 8 levels at factor 1.2, budgets sum to N
    p = oracle.params(y["nFeatures"], y["scaleFactor"], y["nLevels"], y["iniThFAST"],
                      y["minThFAST"])
    t = oracle.tables(p)
    assert sum(int(v) for v in t["nfeat"]) == y["nFeatures"]
