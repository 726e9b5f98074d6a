from .taskpool import Task, Taskpool  # noqa: F401
