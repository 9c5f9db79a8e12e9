"""Time the N=1 drop-in ``sacenv.BoatEnv`` the way main.py drives it (reset, then
step with one action per call, numpy in and out), next to the oracle's N=1 CPU step.
One JSON line. Needs a GPU (the shim has no CPU path)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-agent_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def run(env_step, env_reset, steps, acts):
    env_reset()
    t0 = time.perf_counter()
    for k in range(steps):
        _, _, done, _ = env_step(acts[k % len(acts)])
        if done:
            env_reset()
    return steps / (time.perf_counter() - t0)


def main():
    from sacenv import BoatEnv
    cfg = {"base_settings": {"experiment": 6, "test_mode": 0}}
    np.random.seed(0)
    env = BoatEnv(cfg, None, device="cuda")
    acts = np.random.default_rng(0).uniform(-1, 1, (4096, 1))
    run(env.step, env.reset, 200, acts)                       # warm
    shim = run(env.step, env.reset, 3000, acts)
    from boat_oracle import OracleConfig, OracleVecBoat
    ora = OracleVecBoat(OracleConfig(experiment=6), [0], max_episode_steps=0)

    def ostep(a):
        r = ora.step(np.asarray(a, np.float32).reshape(1))
        return None, None, bool(r["done"][0]), None

    cpu = run(ostep, ora.reset, 3000, acts)
    print(json.dumps({"dropin_boatenv_steps_per_s": shim, "dropin_us_per_step": 1e6 / shim,
                      "oracle_n1_cpu_steps_per_s": cpu, "oracle_us_per_step": 1e6 / cpu,
                      "note": "exp 6, one env, main.py's reset/step loop with numpy actions; the "
                              "reference BoatEnv ran ~75 us/step on one core (BASELINE.md)"}))


if __name__ == "__main__":
    main()
