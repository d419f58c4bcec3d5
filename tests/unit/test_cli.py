"""CLI parity with the reference's distributed_nn.py flags and the method presets."""
import pytest

import ewdml
from ewdml.config import Config, build_parser

REFERENCE_FLAGS = ["--batch-size", "--test-batch-size", "--epochs", "--max-steps", "--lr",
                   "--momentum", "--no-cuda", "--seed", "--log-interval", "--network", "--mode",
                   "--kill-threshold", "--dataset", "--comm-type", "--num-aggregate",
                   "--eval-freq", "--train-dir", "--compress-grad", "--gather-type",
                   "--enable-gpu", "--local_rank"]


def test_every_reference_flag_accepted():
    opts = {o for a in build_parser()._actions for o in a.option_strings}
    for f in REFERENCE_FLAGS:
        assert f in opts, f


def test_reference_defaults():
    c = ewdml.parse_args([])
    assert (c.batch_size, c.test_batch_size, c.epochs, c.max_steps, c.lr, c.momentum) == \
        (128, 500, 100, 10000, 0.01, 0.5)
    assert c.network == "LeNet" and c.dataset == "MNIST" and c.train_dir == "output/models/"


def test_reference_script_invocation():
    # src/run_pytorch_single.sh:4-18
    c = ewdml.parse_args("--lr=0.01 --momentum=0.9 --network=LeNet --dataset=MNIST "
                         "--batch-size=64 --comm-type=Bcast --mode=normal --num-aggregate=2 "
                         "--eval-freq=20 --epochs=10 --max-steps=10000 --train-dir=/tmp/x/ "
                         "--compress-grad=compress --gather-type=gather --enable-gpu= "
                         "--local_rank=0".split())
    assert c.batch_size == 64 and c.enable_gpu is False and c.local_rank == 0


@pytest.mark.parametrize("m,topo,comp,pull,every", [
    (1, "ps", "none", "weights", 1), (2, "ps", "qsgd", "weights", 1),
    (3, "allgather", "none", "grad", 1), (4, "allgather", "qsgd", "grad", 1),
    (5, "allgather", "topk_qsgd", "grad", 1), (6, "allgather", "topk_qsgd", "grad", 20)])
def test_method_presets(m, topo, comp, pull, every):
    c = ewdml.parse_args(["--method", str(m)])
    assert (c.topology, c.compress, c.pull, c.sync_every) == (topo, comp, pull, every)
    assert c.select_best == (m == 6)


def test_compress_grad_none_switch():
    assert ewdml.parse_args(["--compress-grad", "none"]).compress == "none"


def test_ckpt_dir_defaults_to_train_dir():
    assert Config(train_dir="/a/").resolved().ckpt_dir == "/a/"


def test_sync_bn_buffers_alias():
    import ewdml

    assert ewdml.parse_args(["--sync-bn-buffers"]).sync_bn
    assert ewdml.parse_args(["--sync-bn"]).sync_bn
    assert not ewdml.parse_args([]).sync_bn


def test_topology_choices():
    import ewdml

    for t in ("allgather", "ps", "sharded"):
        assert ewdml.parse_args(["--topology", t]).topology == t


def test_error_feedback_brings_its_warmup_recipe():
    import ewdml

    c = ewdml.parse_args(["--compress", "topk_qsgd", "--error-feedback", "--topk-ratio", "0.01"])
    assert c.ef_mode == "dgc"
    assert c.topk_warmup == "0.25,0.125,0.0625,0.03125,0.015625"
    assert c.lr_warmup_epochs == 2.0 and c.lr_warmup_start == 0.1
    c = ewdml.parse_args(["--compress", "topk_qsgd", "--error-feedback", "--ef-warmup", "none"])
    assert c.topk_warmup == "" and c.lr_warmup_epochs == 0
    c = ewdml.parse_args(["--compress", "topk_qsgd", "--error-feedback", "--topk-ratio", "0.4"])
    assert c.topk_warmup == "" and c.lr_warmup_epochs == 0  # nothing denser to warm up from
    c = ewdml.parse_args(["--compress", "topk_qsgd", "--no-error-feedback"])
    assert not c.error_feedback
    assert c.topk_warmup == "" and c.lr_warmup_epochs == 0


def test_error_feedback_is_the_default_for_topk_codecs():
    """Top-k at 1 % without error feedback trains 10-80x slower than dense
    (profiles/validation/ef_stability_r03.md): the CLI turns it on, with its warm-up recipe, for
    the top-k codecs; --no-error-feedback gives the reference's Method 5/6 as published."""
    import ewdml

    for codec in ("topk_qsgd", "topk"):
        c = ewdml.parse_args(["--compress", codec])
        assert c.error_feedback and c.ef_mode == "dgc"
        assert c.topk_warmup and c.lr_warmup_epochs == 2.0
    assert ewdml.parse_args([]).error_feedback  # the default codec is top-k + QSGD
    for codec in ("none", "qsgd", "bf16"):
        assert not ewdml.parse_args(["--compress", codec]).error_feedback
    assert ewdml.parse_args(["--method", "5"]).error_feedback
    assert not ewdml.parse_args(["--method", "5", "--no-error-feedback"]).error_feedback
    assert not ewdml.parse_args(["--method", "3"]).error_feedback


def test_error_feedback_default_only_where_a_residual_is_kept():
    """only the all-gather exchange keeps an error-feedback residual; parameter-server
    and sharded top-k runs default to none and keep the reference's schedule (no EF warm-up)."""
    import ewdml

    for topo in ("ps", "sharded"):
        c = ewdml.parse_args(["--compress", "topk_qsgd", "--topology", topo])
        assert not c.error_feedback
        assert c.topk_warmup == "" and c.lr_warmup_epochs == 0
    c = ewdml.parse_args(["--compress", "topk_qsgd", "--topology", "allgather"])
    assert c.error_feedback and c.topk_warmup


def test_ef21_rejected_at_parse_time_on_the_gpu(monkeypatch):
    """EF21 has only the torch-oracle encode: a GPU run is refused when the configuration is
    parsed, not after the model, buffers and communicator are set up."""
    import ewdml

    assert ewdml.parse_args(["--ef-mode", "ef21", "--device", "cpu"]).ef_mode == "ef21"
    with pytest.raises(ValueError, match="ef21"):
        ewdml.parse_args(["--ef-mode", "ef21", "--device", "cuda"])
    monkeypatch.setenv("EWDML_ORACLE", "1")
    monkeypatch.setenv("EWDML_GRAD_VIEWS", "1")
    assert ewdml.parse_args(["--ef-mode", "ef21", "--device", "cuda"]).ef_mode == "ef21"


def test_wgrad_stream_flag():
    """--wgrad-stream: off by default (the DAG graph's replay cost, profiles/ab/README.md), on /
    auto accepted, anything else rejected."""
    assert ewdml.parse_args([]).wgrad_stream == "off"
    for v in ("on", "auto", "off"):
        assert ewdml.parse_args(["--wgrad-stream", v]).wgrad_stream == v
    with pytest.raises(SystemExit):
        ewdml.parse_args(["--wgrad-stream", "maybe"])


def test_wgrad_stream_is_scoped_to_the_trainer_backward():
    """The side-stream switch is off outside a trainer's backward (so a user's own backward()
    never runs weight gradients on a second stream) and nothing is queued at import."""
    from ewdml.ops import conv as cv

    assert cv._WGRAD_SIDE is False and not cv._SIDE_QUEUE and not cv._SIDE_PENDING
    cv.join_wgrad()  # no-op without side work (no device needed)
