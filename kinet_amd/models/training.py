"""Host-side training glue of the tracking detector (detr_tracking.py:220-283).

Evaluation with targets (not tracking): no track queries -- empty track-query fields
(detr_tracking.py:259-270).  The training two-pass scheme (previous-frame forward without
grad -> Hungarian matching -> track-query sampling -> current-frame forward with grad)
lives here as well once the matcher/criterion land.
"""
import torch


def prepare_track_queries(model, targets):
    if model.training:
        raise NotImplementedError(
            'two-pass track-query training (detr_tracking.py:225-255) is not wired yet; '
            'run tracking mode (model.tracking()) or pass track queries explicitly')
    for target in targets:
        device = target['boxes'].device
        target['track_query_hs_embeds'] = torch.zeros(0, model.hidden_dim).float().to(device)
        target['track_queries_mask'] = torch.zeros(model.num_queries).bool().to(device)
        target['track_queries_fal_pos_mask'] = torch.zeros(model.num_queries).bool().to(device)
        target['track_query_boxes'] = torch.zeros(0, 4).to(device)
        target['track_query_match_ids'] = torch.tensor([]).long().to(device)
