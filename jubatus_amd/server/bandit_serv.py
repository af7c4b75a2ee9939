"""jubabandit glue (reference jubatus/server/server/bandit_serv.cpp:51-110).

register_arm / delete_arm / select_arm / register_reward / get_arm_info /
reset / clear (bandit.idl:17-91); arm_info travels as [trial_count, weight].
"""
from __future__ import annotations

from ..framework.engine_serv import EngineServ
from ..models.bandit import Bandit


class BanditServ(EngineServ):
    type_name = "bandit"

    def uses_gpu(self) -> bool:
        return False

    def build_driver(self, cfg: dict):
        return Bandit(cfg.get("method"), cfg.get("parameter"))

    def register_arm(self, arm_id: str) -> bool:
        self.check_set_config()
        return self.driver.register_arm(arm_id)

    def delete_arm(self, arm_id: str) -> bool:
        self.check_set_config()
        return self.driver.delete_arm(arm_id)

    def select_arm(self, player_id: str) -> str:
        self.check_set_config()
        return self.driver.select_arm(player_id)

    def register_reward(self, player_id: str, arm_id: str, reward: float) -> bool:
        self.check_set_config()
        return self.driver.register_reward(player_id, arm_id, float(reward))

    def get_arm_info(self, player_id: str):
        self.check_set_config()
        return {a: [n, w] for a, (n, w) in self.driver.get_arm_info(player_id).items()}

    def reset(self, player_id: str) -> bool:
        self.check_set_config()
        return self.driver.reset(player_id)
