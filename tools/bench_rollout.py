#!/usr/bin/env python3
"""End-to-end device rollout rate: safelife_amd.rollout.run_agents at the headline
shape (B = 65 536 64x64 prune-still envs, 33x33 packed observations written into the
[T+1, N, 33, 33] states buffer, actions sampled by sl_sample_actions from a
policy's probabilities), followed by sl_gae on the rollout.  The policy here is a
fixed probability table indexed by an integer feature of the observation (no
network): this times the env side of PPO.run_agents + gen_training_batch, not a
model.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "safelife-k2_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps-per-env", type=int, default=20)
    ap.add_argument("--rollouts", type=int, default=5)
    ap.add_argument("--obs", default="packed", choices=["packed", "u8", "bf16"])
    args = ap.parse_args()
    import numpy as np
    import torch
    from safelife_amd import SafeLifeVecEnv, LevelPool
    from safelife_amd.rollout import run_agents, returns_advantages
    dev = torch.device("cuda:0")
    pool = LevelPool.load(os.path.join(REPO, "tests", "golden", "pools", "c3_prune_still_64.npz"))
    ch = None if args.obs == "packed" else tuple(range(15))
    dt = {"packed": "uint16", "u8": "uint8", "bf16": "bfloat16"}[args.obs]
    venv = SafeLifeVecEnv(pool, args.envs, dev, view_shape=(33, 33), output_channels=ch,
                          obs_dtype=dt, penalty_coef=1.0, min_performance=0.01, rng="philox",
                          seed=1234, level_order="random", augment_roll=True)
    table = torch.from_numpy(np.random.RandomState(0).dirichlet(np.ones(9), 16)
                             .astype(np.float32)).to(dev)

    def policy(obs, rnn):
        c = obs[:, 16, 16] if obs.dim() == 3 else obs[:, 16, 16, 0]
        return table[(c.to(torch.int64) & 15)], rnn

    T = args.steps_per_env
    values = torch.zeros((T + 1, args.envs, 1), dtype=torch.float32, device=dev)
    # warm-up: the first reset, and both rollout buffers the loop keeps alive (the
    # previous Rollout is still referenced while the next is allocated; a fresh
    # multi-GB device allocation costs ~0.5 s and is not part of a rollout)
    for _ in range(2):
        ro = run_agents(venv, policy, T)
        returns_advantages(ro.rewards, ro.end_episode, values)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.rollouts):
        ro = run_agents(venv, policy, T)
        ret, adv = returns_advantages(ro.rewards, ro.end_episode, values)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = args.rollouts * T * args.envs
    print(json.dumps({"metric": "run_agents + GAE env-steps/s", "value": round(n / el, 1),
                      "unit": "env-steps/s", "envs": args.envs, "steps_per_env": T,
                      "rollouts": args.rollouts, "obs": args.obs,
                      "ms_per_env_step_batch": round(el / (args.rollouts * T) * 1e3, 4)}))


if __name__ == "__main__":
    main()
