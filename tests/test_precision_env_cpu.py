"""Precision variables of the FaceEmbedder: every accepted word maps to its form, an
unknown word (a typo such as 'fp16x3') raises instead of silently running plain f16, and bench.py's
--precision maps f16x3 / f16c8 onto the ArcFace variable for the FaceEmbedder workloads."""
import os

import pytest

from person_capture_amd import face_embedder as fe
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F16C8, PC_PREC_F16X3, PC_PREC_F32

VARS = ("PERSON_CAPTURE_AMD_PRECISION", "PERSON_CAPTURE_AMD_DET_PRECISION", "PERSON_CAPTURE_AMD_ARC_PRECISION")


@pytest.fixture(autouse=True)
def _clean(monkeypatch):
    for v in VARS:
        monkeypatch.delenv(v, raising=False)


def test_defaults_and_parity_mode(monkeypatch):
    assert fe._precision() == PC_PREC_F16
    assert fe._det_precision() == PC_PREC_F16X3 and fe._arc_precision() == PC_PREC_F16X3
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    assert fe._det_precision() == PC_PREC_F32 and fe._arc_precision() == PC_PREC_F32


@pytest.mark.parametrize("word,want", [("f16", PC_PREC_F16), ("fp32", PC_PREC_F32), ("F16X3", PC_PREC_F16X3),
                                       ("c8", PC_PREC_F16C8)])
def test_arc_words(monkeypatch, word, want):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_ARC_PRECISION", word)
    assert fe._arc_precision() == want


@pytest.mark.parametrize("var,word", [("PERSON_CAPTURE_AMD_ARC_PRECISION", "fp16x3"),
                                      ("PERSON_CAPTURE_AMD_DET_PRECISION", "f16c8"),   # no c8 SCRFD
                                      ("PERSON_CAPTURE_AMD_PRECISION", "f16x3"),       # a mode, not a form
                                      ("PERSON_CAPTURE_AMD_DET_PRECISION", "bf16")])
def test_unknown_words_raise(monkeypatch, var, word):
    monkeypatch.setenv(var, word)
    with pytest.raises(ValueError, match=var):
        fe._det_precision() if "DET" in var else fe._arc_precision()


def test_bench_precision_env(monkeypatch):
    import bench
    bench._precision_env("f16c8")
    assert os.environ["PERSON_CAPTURE_AMD_PRECISION"] == "f16"
    assert fe._arc_precision() == PC_PREC_F16C8 and fe._det_precision() == PC_PREC_F16X3
    assert bench._peak_for("f16x3") == bench.PEAK_F16_TFLOPS and bench._issue_factor("f16x3") == 3.0
