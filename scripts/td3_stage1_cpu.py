"""CPU reproduction of the reference stage-1 TD3 run, one arena at a time like rl/training/train.py, on the kernel
source's host build (tests/hostcheck.py) -- test / diagnostic infrastructure, no GPU.  Usage: python
scripts/td3_stage1_cpu.py <arenas> <episodes> [done|max_steps] [seed]"""
import sys, os, time, json
sys.path[:0] = ["/root/repo/tests", "/root/repo/hockey-env_amd"]
import numpy as np, torch
torch.set_num_threads(4)
from hostcheck import HostTorchEnv, HostVec
from hockey_amd.td3 import TD3Config, train
from hockey_amd.evaluate import reset_params

def host_eval(actor, episodes=100, seed=420, weak=True):
    env = HostVec(episodes, policies=("external", "weak" if weak else "strong"), seed=seed)
    params, max_t, _ = reset_params(episodes, seed)
    env.reset_params(params)
    obs, _ = env.observe()
    live = np.ones(episodes, bool); winner = np.zeros(episodes)
    act = np.zeros((episodes, 8), np.float32)
    for _ in range(max_t + 1):
        with torch.no_grad():
            act[:, :4] = actor(torch.from_numpy(obs)).numpy()
        r = env.step(act)
        d = r.done.astype(bool)
        winner = np.where(live & d, r.info[:, 0], winner)
        live &= ~d
        obs = r.obs
        if not live.any(): break
    env.close()
    return float((winner == 1).mean())

n = int(sys.argv[1]); episodes = int(sys.argv[2]); seed = int(sys.argv[4]) if len(sys.argv) > 4 else 420
cfg = TD3Config.from_json("/root/repo/tests/golden/stage1_config.json", eval_interval=200)
t0 = time.time()
def ev(agent, eps):
    wr = host_eval(agent.actor)
    print(json.dumps({"episode": eps, "updates": agent.train_step, "wr_weak": wr, "t": round(time.time()-t0)}), flush=True)
    return wr
env = HostTorchEnv(n, policies=("external", "external"))
train(n_arenas=n, rounds=episodes // n, cfg=cfg, device="cpu", seed=seed, env=env, eval_fn=ev, graphs=False, episode_end=sys.argv[3] if len(sys.argv) > 3 else "max_steps")
