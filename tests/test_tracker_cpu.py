"""Host logic of kinet_amd.tracker.TrackerKinematic on the CPU (FakeKinetDetector, NMS off so
no kernel runs): each reference defect named in tracker_cfg['reference_defects'] reproduces the
reference's exception at the same step (tracker.py:580-1053), and the fixed
default runs through the same frames."""
import pytest
import torch


def _run(defects=(), enc=False, frames=6, track_thresh=0.8, steps=2):
    from fake_detector import KINEMATIC_CFGS, FakeKinetDetector, kinematic_args, kinematic_blobs
    from kinet_amd.models import DeformablePostProcess
    from kinet_amd.tracker import TrackerKinematic
    cfg = dict(KINEMATIC_CFGS['kinet'], detection_nms_thresh=0.0, track_nms_thresh=0.0,
               track_obj_score_thresh=track_thresh, steps_termination=steps, reference_defects=defects)
    tracker = TrackerKinematic(FakeKinetDetector(n_frames=5, encoded=enc, seed=0), {'bbox': DeformablePostProcess()},
                               cfg, kinematic_args(enc))
    tracker.reset()
    for blob in kinematic_blobs(0, frames):
        tracker.step(blob)
    return tracker


def test_fixed_tracker_runs_on_host():
    t = _run(enc=True, track_thresh=0.99, steps=1)
    assert t.track_num > 0 and t.inactive_tracks and t.frame_index == 6


@pytest.mark.parametrize('defect,exc,kw', [
    ('track_init_confidence_kwarg', TypeError, {}),
    ('metadata_trail_rank', IndexError, {}),
    ('sine_encoding_rank', IndexError, {'enc': True}),
    ('inactive_repeat_method', AttributeError, {'track_thresh': 0.99, 'steps': 1}),
])
def test_reference_defect_switches(defect, exc, kw):
    with pytest.raises(exc):
        _run(defects=(defect,), **kw)


def test_unknown_defect_name_rejected():
    with pytest.raises(ValueError):
        _run(defects=('no_such_defect',))


def test_sine_encoding_matches_reference_layout():
    """The fixed SineEncodingTracklet's (B, n, c*F) output is the reference's (B, n*c*F) output
    (detr_tracking.py:299-307) reshaped: same values, same order."""
    from kinet_amd.tracker import SineEncodingTracklet
    x = torch.rand(3, 5, 4, generator=torch.Generator().manual_seed(0))
    a = SineEncodingTracklet(8)(x)
    b = SineEncodingTracklet(8, reference_rank=True)(x)
    assert a.shape == (3, 5, 32) and b.shape == (3, 160)
    assert torch.equal(a.flatten(1), b)
    assert torch.equal(SineEncodingTracklet(8)(x[0]), a[:1])
