"""Parsing of the native CLIs' console lines (reference formats):

* GPT-2 CLIs: ``[Train] epoch e/E | step s/S (global g/G) | lr .. | loss X | ppl .. | grad_norm .. |
  tokens ..`` (reference gpt2_lora_finetune/main.cpp:627-635);
* Gemma CLI: ``[Step n] Loss=X PPL=.. LR=..`` (reference optim/gemma_trainer.cpp:193-197).

The two regexes are the reference loss plotter's (scripts/Finetune/plot_loss_curve.py:18-19)."""
import re

PLOT_PATTERN1 = r'\[Step (\d+)\] Loss=([\d.]+)'
PLOT_PATTERN2 = r'step (\d+)/\d+.*loss ([\d.]+)'
_GLOBAL = re.compile(r'\(global (\d+)/\d+\).*\| loss ([-\d.naif]+)')
_STEP = re.compile(r'^\[Step (\d+)\] Loss=([-\d.naif]+)')


def native_losses(stdout: str) -> dict:
    """{global step: loss string} from either native line format."""
    out = {}
    for ln in stdout.splitlines():
        m = _GLOBAL.search(ln) if ln.startswith("[Train]") else _STEP.match(ln)
        if m:
            out[int(m.group(1))] = m.group(2)
    return out


def loss_list(stdout: str, as_float: bool = False) -> list:
    d = native_losses(stdout)
    v = [d[k] for k in sorted(d)]
    return [float(x) for x in v] if as_float else v
