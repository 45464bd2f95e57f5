"""The loopz trainer (the reference's default trainer, omniisaacgymenvs/scripts/rlgames_train.py
with algo/ppo/*) on the MI355X kernels of csrc/loopz.hip: same classes, arguments and checkpoint
format (module.Actor / Critic / MLPEncode_wrap / SquashedGaussianDiagonalCovariance, ppo.PPO,
storage.RolloutStorage, vecenv.USVRaisimVecEnv)."""
from .module import Actor, Critic, MLPEncode_wrap, SquashedGaussianDiagonalCovariance  # noqa: F401
from .ppo import PPO  # noqa: F401
from .storage import RolloutStorage  # noqa: F401
from .vecenv import USVRaisimVecEnv  # noqa: F401
