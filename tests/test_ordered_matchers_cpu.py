"""KineT ordered-detection matchers (kinet_amd/models/matcher.py) vs the reference
(matcher.py:13-82, :205-682) on the fixture tests/golden/ordered_matchers.npz (make_golden.py
`ordered_matchers`, reference run on synthetic inputs): identical (prediction, target) index
pairs for Transformer1 / Transformer2 (with and without track queries, with no input
detections), the encoder-only matcher (with / without the empty start token) and
BasicBoxHungarianMatcher (with / without the class cost).  Host logic: runs on the CPU."""
import os

import numpy as np
import pytest
import torch

CASES = ['t1_tracks', 't1_plain', 't2_tracks', 't2_plain', 't2_nodets', 'enc_tracks_empty_start', 'enc_tracks',
         'enc_plain']
KW = dict(cost_class=2.0, cost_bbox=5.0, cost_giou=2.0, focal_loss=True, focal_alpha=0.25, focal_gamma=2.0)
FIELDS = ('boxes', 'labels', 'detections', 'track_query_hs_embeds_meta', 'track_queries_mask', 'track_query_match_ids')


def _load(d, name):
    Qp, div, B, empty_start = d[f'{name}_meta'].tolist()
    out = {'pred_logits': torch.from_numpy(d[f'{name}_pred_logits']),
           'pred_boxes': torch.from_numpy(d[f'{name}_pred_boxes'])}
    tg = [{k: torch.from_numpy(d[f'{name}_{b}_{k}']) for k in FIELDS if f'{name}_{b}_{k}' in d} for b in range(B)]
    return Qp, div, empty_start, out, tg


@pytest.mark.parametrize('name', CASES)
def test_ordered_matchers_match_reference(golden_dir, name):
    from kinet_amd.models import matcher as M
    d = np.load(os.path.join(golden_dir, 'ordered_matchers.npz'))
    Qp, div, empty_start, out, tg = _load(d, name)
    if name.startswith('t1'):
        m = M.OrderDetectionsMatcherTransformer1(Qp, Qp // div, **KW)
    elif name.startswith('t2'):
        m = M.OrderDetectionsMatcherTransformer2(Qp, Qp // div, **KW)
    else:
        m = M.OrderDetectionsMatcherEncoder(use_empty_start=bool(empty_start), **KW)
    res = m(out, tg)
    for b, (p, t) in enumerate(res):
        np.testing.assert_array_equal(p.numpy(), d[f'{name}_{b}_res_pred'])
        np.testing.assert_array_equal(t.numpy(), d[f'{name}_{b}_res_tgt'])


@pytest.mark.parametrize('name,use_class', [('basic', False), ('basic_class', True)])
def test_basic_box_matcher_matches_reference(golden_dir, name, use_class):
    from kinet_amd.models.matcher import BasicBoxHungarianMatcher
    d = np.load(os.path.join(golden_dir, 'ordered_matchers.npz'))
    t, r = BasicBoxHungarianMatcher(use_class=use_class)(
        torch.from_numpy(d[f'{name}_det']), {'boxes': torch.from_numpy(d[f'{name}_boxes']),
                                             'labels': torch.from_numpy(d[f'{name}_labels'])})
    np.testing.assert_array_equal(t.numpy(), d[f'{name}_res_tgt'])
    np.testing.assert_array_equal(r.numpy(), d[f'{name}_res_det'])


def test_encoder_track_pairing_switch(golden_dir):
    """fix_track_pairing=True pairs every track query with the target it carries (the reference
    pairs the reached / not-reached groups crosswise, matcher.py:657-676)."""
    from kinet_amd.models.matcher import OrderDetectionsMatcherEncoder
    d = np.load(os.path.join(golden_dir, 'ordered_matchers.npz'))
    Qp, div, empty_start, out, tg = _load(d, 'enc_tracks_empty_start')
    res = OrderDetectionsMatcherEncoder(use_empty_start=True, fix_track_pairing=True, **KW)(out, tg)
    for (p, t), tgt in zip(res, tg):
        ids = tgt['track_query_match_ids'].tolist()
        K = len(ids)
        for pi, ti in zip(p.tolist()[:K], t.tolist()[:K]):
            assert ids[pi] == ti


def test_build_matcher_ordered():
    from kinet_amd.models.config import load_args
    from kinet_amd.models.matcher import (OrderDetectionsMatcherEncoder, OrderDetectionsMatcherTransformer2,
                                          build_matcher)
    a = load_args('train_kinet', used_ordered_queries=True)
    m = build_matcher(a)
    assert isinstance(m, OrderDetectionsMatcherTransformer2) and m.n_assign == a.num_queries // a.max_number_detection
    assert isinstance(build_matcher(load_args('train_kinet', used_ordered_queries=True, use_encoder_only=True)),
                      OrderDetectionsMatcherEncoder)
