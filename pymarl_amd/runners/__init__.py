from .episode_runner import EpisodeRunner

REGISTRY = {"episode": EpisodeRunner}
