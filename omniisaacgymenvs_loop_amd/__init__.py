"""omniisaacgymenvs_loop_amd: MI355X-native USV CaptureXY env + rl_games PPO hot path.

Drop-in for `task=USV/* train=USV/USV_PPOcontinuous_MLP` of loop-Z/omniisaacgymenvs_loop:
the VecEnvRLGames step()/reset() contract and the rl_games Runner/A2CAgent API,
with the hot path in hand-written HIP (csrc/, C ABI in include/usv_hip.h).
"""
__version__ = "0.1.0"
