from merging_gym.envs.merging_env import MergeEnv, MergeEnvExtend
from merging_gym.envs.vector_env import MergeVecEnv

__all__ = ["MergeEnv", "MergeEnvExtend", "MergeVecEnv"]
