"""Multi-armed bandits (jubabandit): ucb1, epsilon_greedy, softmax, exp3.

Reference: jubatus/server/server/bandit_serv.cpp:51-110 over jubatus_core's
bandit (EXTERNAL); configs config/bandit/*.json. Per player and arm we keep
``arm_info{trial_count, weight}`` (weight = cumulative reward):
* ``register_arm`` / ``delete_arm`` -> False when the arm already exists /
  is unknown; ``register_reward`` -> False for an unknown arm;
* ``select_arm`` with no arm registered raises;
* ``assume_unrewarded``: a selection counts as a trial immediately (a later
  reward only adds weight); otherwise the reward registers the trial;
* ucb1: untried arms first (registration order), then
  argmax mean + sqrt(2 ln(total) / n_i);
* epsilon_greedy (``epsilon``): a uniformly random arm with probability
  epsilon, else the best mean; softmax (``tau``): P(i) ~ exp(mean_i / tau);
* exp3 (``gamma``): P(i) = (1-gamma) w_i / sum w + gamma / K with the
  importance-weighted update w_i *= exp(gamma * (r / P(i)) / K) on reward.

MIX: every server accumulates deltas of (trial_count, weight) per player/arm
and the exp3 log-weights; the mixer sums the deltas cluster-wide and each
server folds the sum into its base (get_diff / mix_diff / put_diff).
"""
from __future__ import annotations

import math
import random
import threading

METHODS = ("ucb1", "epsilon_greedy", "softmax", "exp3")


class BanditError(RuntimeError):
    pass


class Bandit:
    def __init__(self, method: str, parameter: dict | None):
        if method not in METHODS:
            raise ValueError(f"unsupported bandit method: {method}")
        p = dict(parameter or {})
        if "assume_unrewarded" not in p:
            raise ValueError("bandit parameter requires assume_unrewarded")
        self.method = method
        self.assume_unrewarded = bool(p["assume_unrewarded"])
        self.epsilon = float(p.get("epsilon", 0.1))
        self.tau = float(p.get("tau", 0.05))
        self.gamma = float(p.get("gamma", 0.1))
        if method == "epsilon_greedy" and not 0.0 <= self.epsilon <= 1.0:
            raise ValueError("epsilon must be in [0, 1]")
        if method == "softmax" and self.tau <= 0:
            raise ValueError("tau must be positive")
        if method == "exp3" and not 0.0 < self.gamma <= 1.0:
            raise ValueError("gamma must be in (0, 1]")
        self.rng = random.Random(p.get("seed"))
        self._lock = threading.RLock()
        self.arms: list[str] = []
        self.clear()

    def clear(self) -> None:
        with self._lock:
            self.arms = []
            # player -> arm -> [trials, weight]; base (mixed) and local delta
            self.base: dict[str, dict[str, list]] = {}
            self.delta: dict[str, dict[str, list]] = {}
            self.exp3_base: dict[str, dict[str, float]] = {}   # log weights
            self.exp3_delta: dict[str, dict[str, float]] = {}

    # ---------------------------------------------------------------- arms
    def register_arm(self, arm: str) -> bool:
        with self._lock:
            if arm in self.arms:
                return False
            self.arms.append(arm)
            return True

    def delete_arm(self, arm: str) -> bool:
        with self._lock:
            if arm not in self.arms:
                return False
            self.arms.remove(arm)
            for tab in (self.base, self.delta, self.exp3_base, self.exp3_delta):
                for per in tab.values():
                    per.pop(arm, None)
            return True

    def _info(self, player: str, arm: str) -> tuple[int, float]:
        b = self.base.get(player, {}).get(arm, (0, 0.0))
        d = self.delta.get(player, {}).get(arm, (0, 0.0))
        return int(b[0] + d[0]), float(b[1] + d[1])

    def _add(self, player: str, arm: str, trials: int, weight: float) -> None:
        e = self.delta.setdefault(player, {}).setdefault(arm, [0, 0.0])
        e[0] += trials
        e[1] += weight

    def _logw(self, player: str, arm: str) -> float:
        return (self.exp3_base.get(player, {}).get(arm, 0.0)
                + self.exp3_delta.get(player, {}).get(arm, 0.0))

    def _exp3_probs(self, player: str) -> list[float]:
        lw = [self._logw(player, a) for a in self.arms]
        m = max(lw)
        w = [math.exp(x - m) for x in lw]
        s = sum(w)
        k = len(self.arms)
        return [(1.0 - self.gamma) * x / s + self.gamma / k for x in w]

    # -------------------------------------------------------------- select
    def select_arm(self, player: str) -> str:
        with self._lock:
            if not self.arms:
                raise BanditError("select_arm: no arm registered")
            arm = self._choose(player)
            if self.assume_unrewarded:
                self._add(player, arm, 1, 0.0)
            return arm

    def _mean(self, player: str, arm: str) -> float:
        n, w = self._info(player, arm)
        return w / n if n > 0 else 0.0

    def _choose(self, player: str) -> str:
        arms = self.arms
        if self.method == "ucb1":
            infos = [self._info(player, a) for a in arms]
            for a, (n, _) in zip(arms, infos):
                if n == 0:
                    return a
            total = sum(n for n, _ in infos)
            scores = [w / n + math.sqrt(2.0 * math.log(total) / n) for n, w in infos]
            return arms[max(range(len(arms)), key=scores.__getitem__)]
        if self.method == "epsilon_greedy":
            if self.rng.random() < self.epsilon:
                return self.rng.choice(arms)
            means = [self._mean(player, a) for a in arms]
            return arms[max(range(len(arms)), key=means.__getitem__)]
        if self.method == "softmax":
            means = [self._mean(player, a) / self.tau for a in arms]
            m = max(means)
            return self.rng.choices(arms, weights=[math.exp(x - m) for x in means], k=1)[0]
        return self.rng.choices(arms, weights=self._exp3_probs(player), k=1)[0]

    def register_reward(self, player: str, arm: str, reward: float) -> bool:
        with self._lock:
            if arm not in self.arms:
                return False
            if self.method == "exp3":
                p = self._exp3_probs(player)[self.arms.index(arm)]
                d = self.exp3_delta.setdefault(player, {})
                d[arm] = d.get(arm, 0.0) + self.gamma * (reward / p) / len(self.arms)
            self._add(player, arm, 0 if self.assume_unrewarded else 1, float(reward))
            return True

    def get_arm_info(self, player: str) -> dict[str, tuple[int, float]]:
        with self._lock:
            return {a: self._info(player, a) for a in self.arms}

    def reset(self, player: str) -> bool:
        with self._lock:
            for tab in (self.base, self.delta, self.exp3_base, self.exp3_delta):
                tab.pop(player, None)
            return True

    # ----------------------------------------------------------------- MIX
    def get_diff(self) -> dict:
        with self._lock:
            return {"arms": list(self.arms),
                    "info": {p: {a: list(v) for a, v in per.items()} for p, per in self.delta.items()},
                    "exp3": {p: dict(per) for p, per in self.exp3_delta.items()}}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        arms = list(a["arms"]) + [x for x in b["arms"] if x not in a["arms"]]
        info = {p: {k: list(v) for k, v in per.items()} for p, per in a["info"].items()}
        for p, per in b["info"].items():
            tgt = info.setdefault(p, {})
            for k, v in per.items():
                e = tgt.setdefault(k, [0, 0.0])
                e[0] += v[0]
                e[1] += v[1]
        ex = {p: dict(per) for p, per in a["exp3"].items()}
        for p, per in b["exp3"].items():
            tgt = ex.setdefault(p, {})
            for k, v in per.items():
                tgt[k] = tgt.get(k, 0.0) + v
        return {"arms": arms, "info": info, "exp3": ex}

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            for arm in mixed["arms"]:
                if arm not in self.arms:
                    self.arms.append(arm)
            for p, per in mixed["info"].items():
                tgt = self.base.setdefault(p, {})
                for k, v in per.items():
                    e = tgt.setdefault(k, [0, 0.0])
                    e[0] += int(v[0])
                    e[1] += float(v[1])
            for p, per in mixed["exp3"].items():
                tgt = self.exp3_base.setdefault(p, {})
                for k, v in per.items():
                    tgt[k] = tgt.get(k, 0.0) + float(v)
            self.delta = {}
            self.exp3_delta = {}
            return True

    def pack(self) -> dict:
        with self._lock:
            merged = self.mix_diff({"arms": [], "info": {p: {a: list(v) for a, v in per.items()}
                                                         for p, per in self.base.items()},
                                    "exp3": {p: dict(x) for p, x in self.exp3_base.items()}},
                                   self.get_diff())
            return {"method": self.method, **merged}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.clear()
            self.arms = list(obj["arms"])
            self.base = {p: {a: [int(v[0]), float(v[1])] for a, v in per.items()}
                         for p, per in obj["info"].items()}
            self.exp3_base = {p: {a: float(v) for a, v in per.items()} for p, per in obj["exp3"].items()}

    def get_status(self) -> dict[str, str]:
        return {"method": self.method, "num_arms": str(len(self.arms)),
                "num_players": str(len(set(self.base) | set(self.delta)))}
