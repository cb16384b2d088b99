"""The amd-smi source's fast path heals itself: a raw SMU-table
calibration refused by MISMATCH is retried on the sampler thread every
ROCMDASH_SMI_RECALIBRATE_S, and the first retry that matches promotes the source to the
raw path; a refusal of the layout is final. The decision logic is the native
``RawCalibrationPolicy`` (csrc/sources.h) the source runs; each rank's state travels in
its gathered source row and comes out of rank 0's /metrics."""

import numpy as np

from rocmdash.models.schema import SOURCE_FIELDS, SOURCE_INDEX
from rocmdash.prom.exposition import Exposition

S = 1_000_000_000  # ns


def test_mismatch_then_match_promotes(native):
    p = native.RawCalibrationPolicy(60.0)
    assert not p.record(3, 5 * S)  # start-up: 3/8 matched on a busy box -> amd-smi path
    assert not p.raw and p.attempts == 1 and p.last_matched == 3
    assert not p.due(30 * S) and p.due(65 * S)  # retried after the period, not before
    assert not p.record(5, 65 * S)  # still short of 6: stays on amd-smi
    assert not p.due(100 * S) and p.due(125 * S)
    assert p.record(8, 125 * S)  # a quiet minute: promoted
    assert p.raw and p.promotions == 1 and p.attempts == 3
    assert not p.due(10_000 * S)  # never again once raw


def test_startup_match_is_not_a_promotion(native):
    p = native.RawCalibrationPolicy(60.0)
    assert p.record(7, 0) and p.promotions == 0 and not p.due(120 * S)


def test_layout_refusal_is_final(native):
    p = native.RawCalibrationPolicy(60.0)
    assert not p.record(0, 0, True)
    assert p.final_refusal and not p.due(10_000 * S)
    q = native.RawCalibrationPolicy(1.0, need=6)
    q.record(2, 0)
    assert not q.record(8, 2 * S, True) and q.final_refusal  # a final outcome never promotes


class _Src:
    def __init__(self, rows):
        self.last_source = np.array(rows, np.float32)

        class A:
            @staticmethod
            def info_calibration():
                return "amd-smi matched 8/8 (interconnect 8, xcd 8; >= 6 needed) [attempt 3]"

        self.agent = A()


def test_metrics_carry_every_gpus_fast_path():
    from rocmdash.serve import _export_sources

    def row(raw, att, matched, promo):
        r = np.full(len(SOURCE_FIELDS), np.nan, np.float32)
        r[SOURCE_INDEX["smi_raw_path"]] = raw
        r[SOURCE_INDEX["smi_calibration_attempts"]] = att
        r[SOURCE_INDEX["smi_calibration_matched"]] = matched
        r[SOURCE_INDEX["smi_calibration_promotions"]] = promo
        r[SOURCE_INDEX["smi_calibration_final"]] = 0
        return r

    synthetic = np.full(len(SOURCE_FIELDS), np.nan, np.float32)
    exp = Exposition()
    _export_sources(exp, _Src([row(1, 3, 8, 1), row(0, 2, 4, 0), synthetic]), ["0", "1", "2"])
    text = exp.text()
    assert 'rocmdash_smi_raw_path{gpu_id="0"} 1' in text and 'rocmdash_smi_raw_path{gpu_id="1"} 0' in text
    assert 'gpu_id="2"' not in text  # a synthetic source has no fast path
    assert 'rocmdash_smi_calibration_promotions_total{gpu_id="0"} 1' in text
    assert 'rocmdash_smi_calibration_matched{gpu_id="1"} 4' in text
    assert "rocmdash_smi_calibration_info{" in text and "[attempt 3]" in text
