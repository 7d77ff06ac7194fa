import pytest

from rocfm.config import Config, parse_flags, str2bool


def test_reference_flag_defaults():
    c = Config()
    assert c.embedding_size == 32 and c.batch_size == 64 and c.learning_rate == 0.0005
    assert c.deep_layers == "256,128,64" and c.dropout == "0.5,0.5,0.5" and c.optimizer == "Adam"
    assert c.layers == [256, 128, 64] and c.keep_probs == [0.5, 0.5, 0.5]


def test_notebook_hyperparameters_parse():
    # NB-PS:82-93 style command line, incl. an undefined flag (perform_shuffle) and "--flag False"
    argv = ["--deep_layers", "128,64,32", "--batch_size", "1024", "--feature_size", "117581", "--field_size", "39",
            "--num_epochs", "10", "--log_steps", "10", "--perform_shuffle", "0", "--enable_s3_shard", "False",
            "--training_channel_name", "training", "--unknown_flag", "x"]
    c = parse_flags(argv)
    assert c.layers == [128, 64, 32] and c.batch_size == 1024 and c.feature_size == 117581
    assert c.enable_s3_shard is False and c.perform_shuffle is False
    c.validate()


@pytest.mark.parametrize("argv,val", [(["--batch_norm"], True), (["--nobatch_norm"], False),
                                      (["--batch_norm=False"], False), (["--batch_norm", "True"], True),
                                      (["--batch_norm", "0"], False), (["--batch_norm=yes"], True)])
def test_strict_bool_forms(argv, val):
    assert parse_flags(argv).batch_norm is val


def test_str2bool_rejects_garbage():
    with pytest.raises(ValueError):
        str2bool("maybe")


def test_validation_errors():
    c = parse_flags(["--feature_size", "10", "--field_size", "3", "--deep_layers", "8,4", "--dropout", "0.5"])
    with pytest.raises(ValueError):
        c.validate()
    c = parse_flags(["--feature_size", "10", "--field_size", "3", "--optimizer", "SGD2"])
    with pytest.raises(ValueError):
        c.validate()


def test_config_file(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("batch_size: 256\noptimizer: Adagrad\nbatch_norm: true\n")
    c = parse_flags(["--config", str(p), "--batch_size", "128"])
    assert c.batch_size == 128 and c.optimizer == "Adagrad" and c.batch_norm is True
