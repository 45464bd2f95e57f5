"""rl_games Runner (rl_games/rl_games/torch_runner.py:45-144): same load()/run()
contract, algo 'a2c_continuous' -> A2CAgent, player 'a2c_continuous' ->
PpoPlayerContinuous; model 'continuous_a2c_logstd' + network
'actor_critic_mlp_dict' are the only ones on the USV path."""
from __future__ import annotations

import copy
import os
import random
from typing import Any, Dict

import numpy as np
import torch

from .a2c_continuous import A2CAgent
from .players import PpoPlayerContinuous


class Runner:
    def __init__(self, algo_observer=None):
        self.algo_factory = {"a2c_continuous": lambda **kw: A2CAgent(**kw)}
        self.player_factory = {"a2c_continuous": lambda **kw: PpoPlayerContinuous(**kw)}
        self.algo_observer = algo_observer
        self.params = None

    def reset(self):
        pass

    def load_config(self, params: Dict[str, Any]) -> None:
        self.seed = int(params.get("seed", 42))
        if params["config"].get("multi_gpu", False):
            self.seed += int(os.getenv("LOCAL_RANK", "0"))        # torch_runner.py:74-75
        torch.manual_seed(self.seed)
        np.random.seed(self.seed)
        random.seed(self.seed)
        params["seed"] = self.seed
        if params["algo"]["name"] not in self.algo_factory:
            raise NotImplementedError(f"algo {params['algo']['name']}")
        if params["model"]["name"] != "continuous_a2c_logstd":
            raise NotImplementedError(f"model {params['model']['name']} is not on the USV hot path")
        if params["network"]["name"] != "actor_critic_mlp_dict":
            raise NotImplementedError(f"network {params['network']['name']} is not on the USV hot path")
        net = params["network"]
        if list(net["mlp"]["units"]) != [128, 128] or net["mlp"]["activation"] != "tanh" or net.get("separate"):
            raise NotImplementedError("kernels implement the shared tanh MLP 33-128-128 (USV_PPOcontinuous_MLP)")
        if not net["space"]["continuous"].get("fixed_sigma", True):
            raise NotImplementedError("fixed_sigma=False is not on the USV hot path")
        config = params["config"]
        config.setdefault("features", {})
        config["features"]["observer"] = self.algo_observer
        self.params = params

    def load(self, yaml_config: Dict[str, Any]) -> None:
        config = copy.deepcopy(yaml_config)
        self.default_config = copy.deepcopy(config["params"])
        self.load_config(params=copy.deepcopy(config["params"]))

    def run_train(self, args: Dict[str, Any]):
        print("Started to train")
        agent = self.algo_factory[self.params["algo"]["name"]](base_name="run", params=self.params)
        checkpoint = args.get("checkpoint")
        if checkpoint:
            agent.restore(checkpoint)
        return agent.train()

    def run_play(self, args: Dict[str, Any]):
        print("Started to play")
        player = self.player_factory[self.params["algo"]["name"]](params=self.params)
        if args.get("checkpoint"):
            player.restore(args["checkpoint"])
        return player.run()

    def create_player(self):
        return self.player_factory[self.params["algo"]["name"]](params=self.params)

    def run(self, args: Dict[str, Any]):
        if args.get("train"):
            return self.run_train(args)
        if args.get("play"):
            return self.run_play(args)
        return self.run_train(args)
