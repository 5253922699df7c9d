"""The reference's OWN training loop on the restated physics, on the CPU ("find the cause").

Question: when the GPU TD3 loop (hockey_amd.td3.train) trained from scratch plateaus in most seeds, is that the loop or
the task?  This runs the reference's unmodified learning code -- rl/td3/agent.py TD3Agent (networks, Adam, noise,
annealing, random phase), rl/td3/learner.py TD3Learner, rl/replay/uniform_buffer.py, rl/training/opponent_manager.py
with the reference's own BasicOpponent (hockey/hockey_env.py:781-833), rl/training/train.py TD3Trainer (episode loop,
32 updates per episode, evaluation cadence) and rl/utils/evaluator.py Evaluator -- imported from /root/reference in
this build container, with only the environment swapped: HockeyEnv's step / reset / obs_agent_two are the C oracle
(oracle/hk_oracle.c, the restatement the GPU kernel equals bit for bit; reset placement by hockey_amd.placement, the
G1-pinned restatement of hockey_env.py:345-418).  Box2D and gymnasium are absent here, so the
reference's hockey_env module is imported with the stub modules of tests/golden/make_golden.py, only for
BasicOpponent.

Harness changes (not learning code): TD3Trainer._run_episode ends an episode at done when ``--episode-end done`` (the
semantics behind the recorded metrics: their returns never exceed +10; the current file steps 500 times),
and _maybe_evaluate keeps the evaluation and ModelManager's best rule (score min(WR_strong, WR_weak) > best + 0.01)
but writes JSON instead of checkpoint files and matplotlib plots.  Build container only; nothing here ships.

Usage: python scripts/reference_loop_study.py --noise gaussian --seed 42 [--episodes 10000] --out <json>
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path[:0] = [os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from hockey_amd.placement import np_random, placement  # noqa: E402

NOISES = {"gaussian": "gaussian", "ou": "ornstein-uhlenbeck", "pink": "pink", "uniform": "uniform"}


def reference_modules():
    import make_golden

    make_golden.install_stubs()
    sys.path.insert(0, REF)
    import logging

    from rl.utils.logger import Logger
    lg = logging.getLogger("RL-quiet")
    lg.addHandler(logging.NullHandler())
    lg.propagate = False
    Logger._logger = lg  # the reference logs every few thousand steps; keep the study's stdout readable
    import hockey.hockey_env as H
    from rl.td3.agent import TD3Agent
    from rl.td3.config import TD3Config
    from rl.training.train import TD3Trainer
    from rl.utils.evaluator import Evaluator
    return H, TD3Agent, TD3Config, TD3Trainer, Evaluator


class Box:
    def __init__(self, low, high, shape):
        self.shape = shape
        self.low = np.full(shape, low, np.float32)
        self.high = np.full(shape, high, np.float32)


class OracleHockeyEnv:
    """HockeyEnv (NORMAL mode, keep_mode) with the C oracle as its world: the surface rl/ uses."""

    def __init__(self):
        self.world = O.OracleWorld(True, 0)
        self.observation_space = Box(-np.inf, np.inf, (18,))
        self.action_space = Box(-1.0, 1.0, (8,))
        self.one_starts = True
        self.unwrapped = self
        self.reset(one_starting=True)

    def reset(self, one_starting=None, seed=None, options=None):  # hockey_env.py:345-418, NORMAL mode
        self.one_starts = bool(one_starting) if one_starting is not None else (not self.one_starts)
        rng, _ = np_random(seed)
        params, max_t = placement(0, self.one_starts, rng)
        self.world.reset(params, max_t)
        return self.world.obs().astype(np.float64), {}

    def step(self, action):
        a = np.clip(np.asarray(action, np.float64), -1, 1).astype(np.float32)
        obs, r, done, info, _ = self.world.step(a)
        return obs.astype(np.float64), float(r), bool(done), False, {
            "winner": int(info[0]), "reward_closeness_to_puck": float(info[1]), "reward_touch_puck": float(info[2]),
            "reward_puck_direction": float(info[3])}

    def obs_agent_two(self):
        return self.world.obs_two().astype(np.float64)


class OracleHockeyOne(OracleHockeyEnv):
    """HockeyEnv_BasicOpponent (hockey_env.py:875-886) with the reference's own BasicOpponent."""

    def __init__(self, H, weak):
        self.opponent = H.BasicOpponent(weak=weak)
        super().__init__()
        self.action_space = Box(-1.0, 1.0, (4,))

    def step(self, action):
        a2 = self.opponent.act(self.obs_agent_two())
        return super().step(np.hstack([action, a2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--noise", choices=sorted(NOISES), default="gaussian")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--curriculum", default="noise_study")
    ap.add_argument("--protocol", choices=["scratch", "stage1", "stage2", "sp_per"], default="scratch",
                    help="stage2: the report's Stage II setup (definitions.py:93-114): resume from the stage-1 best "
                         "checkpoint, curriculum stage2, lr 3e-4, noise floor 0.06 (as scripts/noise_study.py); "
                         "sp_per: the baseline row of prioritized_selfplay_study (definitions.py:34-66): resume, "
                         "curriculum ablation, OU noise, no PER, no self-play, config.py defaults otherwise; stage1: "
                         "definitions.py:70-90, from scratch on the weak-bot curriculum")
    ap.add_argument("--final-games", type=int, default=1000)
    ap.add_argument("--episode-end", choices=["done", "max_steps"], default="done")
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    H, TD3Agent, TD3Config, TD3Trainer, Evaluator = reference_modules()
    from rl.experiment.tracking import set_global_seed

    set_global_seed(args.seed)  # rl/main.py:86
    cfg = TD3Config()
    over = dict(curriculum_name=args.curriculum, noise_mode=NOISES[args.noise], prioritized_replay=False,
                use_self_play=False, use_noise_annealing=True)  # definitions.py:10-31 noise_study
    if args.protocol == "stage2":
        over.update(curriculum_name="stage2", lr_q=3e-4, lr_pol=3e-4, noise_min_scale=0.06)
    if args.protocol == "sp_per":
        over.update(curriculum_name="ablation", noise_mode=NOISES["ou"])
    if args.protocol == "stage1":  # definitions.py:70-90 (lr 4e-4 is config.py's default)
        over.update(curriculum_name="stage1", lr_q=4e-4, lr_pol=4e-4)
    for k, v in over.items():
        setattr(cfg, k, v)
    train_env = OracleHockeyEnv()
    evaluators = {"strong": Evaluator(OracleHockeyOne(H, False), episodes=cfg.eval_episodes),
                  "weak": Evaluator(OracleHockeyOne(H, True), episodes=cfg.eval_episodes)}
    agent = TD3Agent(env=train_env, config=cfg, h=256, max_total_steps=args.episodes * cfg.max_steps, seed=args.seed)
    if args.protocol not in ("scratch", "stage1"):  # agent.load (rl/td3/agent.py:278-286), read weights-only
        ck = torch.load(os.path.join(REF, "pretrained", "stage_1", "models", "td3_best.pt"), map_location="cpu",
                        weights_only=True)
        for key, net in (("policy", agent.policy), ("critic", agent.critic), ("target_policy", agent.target_policy),
                         ("target_critic", agent.target_critic)):
            net.load_state_dict(ck[key])
    out = {"study": "reference rl/ loop on the oracle", "protocol": args.protocol, "noise": args.noise,
           "seed": args.seed, "episodes": args.episodes, "curriculum": cfg.curriculum_name,
           "episode_end": args.episode_end, "evals": [], "best": None}
    t0 = time.time()
    best = {"score": float("-inf")}

    class Trainer(TD3Trainer):
        def _run_episode(self):  # rl/training/train.py:135-172, with the recorded runs' break at done
            if args.episode_end == "max_steps":
                return super()._run_episode()
            obs, _ = self.train_env.reset(seed=self.agent.seed + self.current_episode)
            self.agent.reset()
            if self.opponent_manager is not None:
                self.opponent_manager.step()
            ep_reward, steps = 0, 0
            for _ in range(self.max_steps):
                action1 = self.agent.get_action(obs, noise=True)
                obs2 = self.train_env.unwrapped.obs_agent_two()
                action2 = self.opponent_manager.select_action(obs2)
                next_obs, reward, done, trunc, _ = self.train_env.step(np.concatenate([action1, action2]))
                self.agent.replay_buffer.push(obs, action1, reward, next_obs, done or trunc)
                ep_reward += reward
                obs = next_obs
                steps += 1
                if done or trunc:
                    if self.opponent_manager is not None:
                        self.opponent_manager.register_outcome(1 if reward > 0 else 0)
                    break
            return ep_reward, steps

        def _maybe_evaluate(self, ep):  # rl/training/train.py:210-248 without files and plots
            if ep % self.eval_interval != 0:
                return
            wr_s, r_s = self.evaluators["strong"].evaluate(self.agent)
            wr_w, r_w = self.evaluators["weak"].evaluate(self.agent)
            score = min(wr_s, wr_w)
            rec = {"episode": ep, "wr_strong": wr_s, "wr_weak": wr_w, "r_strong": r_s, "r_weak": r_w, "score": score,
                   "total_steps": self.agent.total_steps, "noise_scale": self.agent.current_noise_scale,
                   "wall_s": round(time.time() - t0, 1)}
            if score > best["score"] + 0.01:  # rl/utils/model_manager.py:15-23
                best["score"] = score
                best["state"] = {k: v.detach().clone() for k, v in self.agent.policy.state_dict().items()}
                out["best"] = dict(rec)
            out["evals"].append(rec)
            with open(args.out, "w") as f:
                json.dump(out, f, indent=1)
            print(json.dumps(rec), flush=True)

        def _save_checkpoint(self):
            pass

    tr = Trainer(agent=agent, train_env=train_env, evaluators=evaluators, model_dir=os.path.join("/tmp", "reflooprun"),
                 metrics_dir=os.path.join("/tmp", "reflooprun"), plot_dir=os.path.join("/tmp", "reflooprun"),
                 max_episodes=args.episodes)
    tr.train()
    if "state" in best:  # the best checkpoint re-evaluated on fresh placements (as scripts/noise_study.py)
        agent.policy.load_state_dict(best["state"])
        seed0 = agent.seed
        agent.seed = 100_000
        fin = {"games": args.final_games}
        for opp in ("strong", "weak"):
            wr, rr = Evaluator(OracleHockeyOne(H, opp == "weak"), episodes=args.final_games).evaluate(agent)
            fin[f"wr_{opp}"], fin[f"r_{opp}"] = wr, rr
        agent.seed = seed0
        out["final_eval"] = fin
    out["wall_s"] = round(time.time() - t0, 1)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
