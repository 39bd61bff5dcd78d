"""Ray-compatible training executor for the raytrain chart (no Ray cluster on a single
MI355X node): ``mxtrain.raylike.train`` mirrors ``ray.train`` (TorchTrainer, ScalingConfig,
RunConfig, report, get_context, Checkpoint) and ``mxtrain.raylike.lightning`` a minimal
Lightning-style loop with the ``ray.train.lightning`` hooks."""


def init(*args, **kwargs):
    """`ray.init()` equivalent: the worker group is local, nothing to connect to."""
    return None


def is_initialized() -> bool:
    return True


def shutdown():
    return None
