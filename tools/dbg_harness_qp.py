import os, sys
ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from ccmpc import planner, harness, standins
import test_gpu_harness as T
gpu = torch.device("cuda", 0)
scen = T._scenario(gpu, False)
stats = scen.episode(0)
steps = scen.steps
for trial in range(2):
    ref_agent = planner.MidlevelAgent(prediction_horizon=8, n_ideal=T.N_IDEAL, device=gpu)
    for j, s in enumerate(steps):
        sp, an, to = ref_agent.compute_prediction_controls(
            s["frame"], s["T"], s["shrinking"], s["sampler"], s["minpos"], s["pasts"],
            s["x_init"], s["goal"], s["ref"], s["bboxes"])
        rec_same = ref_agent.last_records.tobytes() == s["records"].tobytes()
        du = np.abs(ref_agent.last_ctrl["u"] - s["U_star"].T.ravel()).max() if "U_star" in s else None
        print(trial, j, s["T"], "rec", rec_same, "dspeed", float(np.abs(sp - s["speeds"]).max()),
              "dX", float(np.abs(ref_agent.last_ctrl["X_star"] - s["X_star"]).max()),
              "x_init", s["x_init"][:2], flush=True)
