"""The reference's prediction module (collect/in_simulation/midlevel/prediction.py) at the
boundary the planner calls it: generate_vehicle_latents and Trajectron++'s
prediction_output_to_trajectories, which MidlevelAgent.do_prediction (v8ideal/__init__.py:
414-467) runs when its eval_stg is a real Trajectron++ model (no sample_boundary).

Everything here is host glue around Trajectron++'s own model objects (the encoder, p(z|x),
the latent sampler and the GRU decoder live in eval_stg); the product path starts where the
5-tuple ends: make_ovehicles' bucketing, the generators and the QP run on the GPU from
predictions + z (ccmpc_bucket_predictions -> ..., step.StepGraph with source="predictions").  Trajectron++ is an un-vendored submodule (absent here), so its imports
are lazy and fail the way the reference's module import does.
"""
import numpy as np


def _trajectron():
    try:
        from model.dataset import get_timesteps_data          # trajectron-plus-plus/trajectron
        from model.model_utils import ModeKeys
    except ModuleNotFoundError as e:                         # prediction.py:13-17
        raise Exception("You forgot to link trajectron-plus-plus/trajectron") from e
    return get_timesteps_data, ModeKeys


def generate_vehicle_latents(eval_stg, scene, timesteps, num_samples=200, ph=8, z_mode=False,
                             gmm_mode=False, full_dist=False, all_z_sep=False,
                             keep_on_device=False):
    """prediction.py:19-105: one batch of the scene's VEHICLE nodes at `timesteps` through
    eval_stg's node model -- p(z|x), sample_p, p_y_xz -- returned as the reference returns it:

      z               (nodes, num_samples) int64, the argmax of each one-hot latent sample
      predictions     (nodes, num_samples, ph, 2) float32, scene-relative positions
      nodes           the batch's nodes (the ego's included; make_ovehicles skips it)
      predictions_dict {timestep: {node: (1, num_samples, ph, 2)}}
      latent_probs    (nodes, n_latent) p(z|x)

    keep_on_device (not in the reference, opt-in): z and predictions stay torch tensors on
    eval_stg.device -- the same values (the argmax of a one-hot sample is its one index, so
    torch's and numpy's agree), laid out as the numpy route lays them out -- and
    predictions_dict holds views of them.  The only consumer is make_ovehicles' bucketing,
    which runs on the same GPU (v8ideal/__init__.py:469-505: the arrays are only indexed by z),
    so the particles never cross PCIe."""
    get_timesteps_data, ModeKeys = _trajectron()
    node_type = eval_stg.env.NodeType.VEHICLE
    if node_type not in eval_stg.pred_state:
        raise Exception("fail")
    model = eval_stg.node_models_dict[node_type]
    batch = get_timesteps_data(env=eval_stg.env, scene=scene, t=timesteps, node_type=node_type,
                               state=eval_stg.state, pred_state=eval_stg.pred_state,
                               edge_types=model.edge_types, min_ht=1, max_ht=eval_stg.max_ht,
                               min_ft=0, max_ft=0, hyperparams=eval_stg.hyperparams)
    if batch is None:
        raise Exception("fail")
    (first_history_index, x_t, _, x_st_t, _, neighbors_data_st, neighbors_edge_value,
     robot_traj_st_t, map_), nodes, timesteps_o = batch
    dev = eval_stg.device
    if robot_traj_st_t is not None:
        robot_traj_st_t = robot_traj_st_t.to(dev)
    if hasattr(map_, "to"):
        map_ = map_.to(dev)
    mode = ModeKeys.PREDICT
    x, x_nr_t, _, y_r, _, n_s_t0 = model.obtain_encoded_tensors(
        mode=mode, inputs=x_t.to(dev), inputs_st=x_st_t.to(dev), labels=None, labels_st=None,
        first_history_indices=first_history_index, neighbors=neighbors_data_st,
        neighbors_edge_value=neighbors_edge_value, robot=robot_traj_st_t, map=map_)
    model.latent.p_dist = model.p_z_x(mode, x)
    latent_probs = np.squeeze(model.latent.get_p_dist_probs().cpu().detach().numpy())
    z, n_samples, n_components = model.latent.sample_p(
        num_samples, mode, most_likely_z=z_mode, full_dist=full_dist, all_z_sep=all_z_sep)
    _, predictions = model.p_y_xz(mode, x, x_nr_t, y_r, n_s_t0, z, ph, n_samples,
                                  n_components, gmm_mode)
    if keep_on_device:
        import torch
        z = torch.argmax(z.detach(), dim=-1).transpose(0, 1).contiguous()   # (nodes, samples)
        predictions = predictions.detach().to(torch.float32)
        pd = {}
        for i, ts in enumerate(timesteps_o):
            pd.setdefault(ts, {})[nodes[i]] = predictions[:, i:i + 1].transpose(0, 1)
        return z, predictions.transpose(0, 1).contiguous(), nodes, pd, latent_probs
    z = z.cpu().detach().numpy()                    # (samples, nodes, n_latent) one-hot
    predictions = predictions.cpu().detach().numpy()  # (samples, nodes, ph, 2)
    predictions_dict = {}
    for i, ts in enumerate(timesteps_o):
        predictions_dict.setdefault(ts, {})[nodes[i]] = np.transpose(predictions[:, [i]],
                                                                     (1, 0, 2, 3))
    return (np.swapaxes(np.argmax(z, axis=-1), 0, 1), np.swapaxes(predictions, 0, 1), nodes,
            predictions_dict, latent_probs)


def prediction_output_to_trajectories(prediction_output_dict, dt, max_h, ph, map=None,
                                      prune_ph_to_future=False):
    """Trajectron++'s utils.prediction_output_to_trajectories (called at v8ideal/__init__.py:
    449-455): per timestep t and node, the prediction as given, the history (steps t - max_h
    .. t, current position included) and the future (t + 1 .. t + ph) positions from the
    node's own track (node.get(range, {'position': ['x', 'y']})), rows with a NaN (outside the
    track) dropped.  Returns (output_dict, histories_dict, futures_dict)."""
    state = {"position": ["x", "y"]}
    out, hist, fut = {}, {}, {}
    for t, per_node in prediction_output_dict.items():
        out[t], hist[t], fut[t] = {}, {}, {}
        for node, pred in per_node.items():
            h = node.get(np.array([t - max_h, t]), state)
            h = h[~np.isnan(h.sum(axis=1))]
            f = node.get(np.array([t + 1, t + ph]), state)
            f = f[~np.isnan(f.sum(axis=1))]
            if prune_ph_to_future:
                pred = pred[:, :, :f.shape[0]]
                if pred.shape[2] == 0:
                    continue
            if map is not None:
                h, f, pred = map.to_map_points(h), map.to_map_points(f), map.to_map_points(pred)
            out[t][node], hist[t][node], fut[t][node] = pred, h, f
    return out, hist, fut
