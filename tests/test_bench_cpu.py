"""bench.py host logic without a GPU: defaults of the measurement flags, the two-stream
region's memory check (no device -> no second batch), and the step functions."""
import bench
import tkz
from tkz import synth


def test_bench_defaults():
    a = bench.parse_args([])
    assert a.gpus == 1 and a.config == 1 and a.streams == 1
    assert not a.no_pipelined_run and not a.no_memo_off_run and not a.no_cpu_baseline


def test_two_batches_fit_without_device():
    """tkz_dev_mem_info fails without a GPU: the pipelined region is skipped, not guessed."""
    tok = tkz.Tokenizer.from_json(synth.tokenizer_json(0))
    assert bench.two_batches_fit(tok, 1 << 20, 1000) is False


def test_stream_steps_single_batch():
    """One batch runs on the tokenizer's own stream (no HIP stream is created)."""

    class FakeBatch:
        def __init__(self):
            self.runs = self.syncs = 0

        def run(self, stream=None):
            self.runs += 1

        def sync(self):
            self.syncs += 1

    b = FakeBatch()
    step, sync = bench.stream_steps(tkz, [b])
    step(), step(), sync()
    assert (b.runs, b.syncs) == (2, 1)
