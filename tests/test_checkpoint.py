"""Checkpoint / resume of the bundled MNIST workload (SURVEY §5 checkpoint row: the reference has
none; its workloads' checkpoints would go to --data volumes). A run interrupted at step 20 and
resumed from its checkpoint must end bit-identical to an uninterrupted 30-step run: parameters,
Adam state, epoch order and shuffle generator are all in the checkpoint (CPU path)."""
import torch

from arena_amd.examples import mnist


def test_resume_is_bit_exact(tmp_path):
    common = ["--n_train", "1000", "--device", "cpu", "--eval_every", "10",
              "--log_dir", str(tmp_path / "tb"), "--hidden", "64"]
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    assert mnist.main(["--max_steps", "30", "--checkpoint", a] + common) == 0
    assert mnist.main(["--max_steps", "20", "--checkpoint", b] + common) == 0   # 2 epochs
    assert torch.load(b, weights_only=True)["step"] == 20
    assert mnist.main(["--max_steps", "30", "--checkpoint", b] + common) == 0   # resume
    sa, sb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    assert sa["step"] == sb["step"] == 30
    for k in ("P", "M", "V", "perm"):
        assert torch.equal(sa[k], sb[k]), k
