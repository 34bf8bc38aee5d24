"""ORACLE TOOLING ONLY — minimal stand-in for gym 0.25.2's surface that
/root/reference/torch_impl/env imports (env.py:3-5, wrappers.py:1-3), so that
oracle/gen_golden.py can import the reference in the build container to
produce golden fixtures.  Never used by the product or on the GPU box."""
from . import spaces  # noqa: F401


class Env:
    pass


class Wrapper:
    def __init__(self, env, new_step_api=False):
        self.env = env
        self._observation_space = None

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def action_space(self):
        return self.env.action_space

    @property
    def observation_space(self):
        return self._observation_space

    @observation_space.setter
    def observation_space(self, v):
        self._observation_space = v

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, a):
        return self.env.step(a)


class ObservationWrapper(Wrapper):
    def reset(self, **kw):
        return self.observation(self.env.reset(**kw))

    def step(self, a):
        o, r, term, trunc, info = self.env.step(a)
        return self.observation(o), r, term, trunc, info
