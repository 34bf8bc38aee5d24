"""ORACLE TOOLING ONLY — empty stand-in so oracle/gen_evaluator_golden.py can
import torch_impl/agents/dqn.py, whose `import matplotlib.pyplot as plt`
(dqn.py:7) serves plotting helpers the evaluation path never calls.
matplotlib is not installed in this image."""
