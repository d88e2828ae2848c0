"""SVM prediction of predict mode's Output (f3): SVMPredict
(libsvm/svm_util.cpp:41-95) over libsvm 2.8x, restated in
csrc/host/svm_predict.cpp (sk_svm_model_load / sk_svm_predict).

The models are trained by scikit-learn's libsvm on precomputed kernels and
written in libsvm's model text; labels and decision values are pinned
against scikit-learn's own predictions (the published libsvm algorithm),
probabilities against the oracle restatement of the reference's pairwise
coupling (oracle/svm_oracle.py; scikit-learn's newer libsvm only agrees to
its 0.005/k stopping tolerance).  CPU only."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import svm_oracle as so

sklearn_svm = pytest.importorskip("sklearn.svm")


def _kernel(a, b):
    d = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
    return np.exp(-d / 4.0)


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(0x5EED0A00)
    X = rng.normal(size=(48, 4))
    T = rng.normal(size=(12, 4))
    y3 = np.where(X[:, 0] > 0.4, 3, np.where(X[:, 1] > 0, 1, -1))
    y2 = np.where(X[:, 0] + 0.5 * X[:, 2] > 0, 1, -1)
    return _kernel(X, X), _kernel(T, X), y2, y3, X[:, 0] - X[:, 1] ** 2


def _model_of(clf, svm_type, classes=None):
    # scikit-learn keeps libsvm's own coefficients and intercepts in the
    # private _dual_coef_ / _intercept_ (its public ones are sign-flipped for
    # two classes); libsvm's rho = -intercept
    m = dict(svm_type=svm_type, sv_index=(clf.support_ + 1).tolist(),
             sv_coef=np.atleast_2d(clf._dual_coef_).tolist(), rho=(-np.ravel(clf._intercept_)).tolist())
    if classes is not None:
        m.update(nr_class=len(classes), label=[int(c) for c in classes], nSV=clf.n_support_.tolist())
        if getattr(clf, "probability", False):
            m.update(probA=np.ravel(clf.probA_).tolist(), probB=np.ravel(clf.probB_).tolist())
    else:
        m.update(nr_class=2)
    return m


@pytest.mark.parametrize("which", ["binary", "three"])
def test_c_svc_probability_and_decision(tmp_path, data, which):
    K, Kt, y2, y3, _ = data
    y = y2 if which == "binary" else y3
    clf = sklearn_svm.SVC(kernel="precomputed", C=2.0, probability=True, random_state=0,
                          decision_function_shape="ovo").fit(K, y)
    m = _model_of(clf, "c_svc", clf.classes_)
    path = tmp_path / "model"
    so.write_model(path, m)
    model = ska.SVMModel(path)
    assert model.svm_type == 0 and model.nr_class == len(clf.classes_) and model.has_probability
    assert model.labels == [int(c) for c in clf.classes_]
    ref_dec = clf.decision_function(Kt)
    if which == "binary":
        ref_dec = -ref_dec[:, None]  # scikit-learn flips libsvm's sign for two classes
    for t in range(Kt.shape[0]):
        lab, dec = model.predict(Kt[t], cnt=t + 1, probability=False)
        assert lab == clf.predict(Kt[t:t + 1])[0]
        assert np.allclose(dec, ref_dec[t], rtol=1e-10, atol=1e-12)
        assert np.allclose(dec, so.decision_values(m, Kt[t]), rtol=1e-13, atol=1e-14)
        lab_p, prob = model.predict(Kt[t], cnt=t + 1, probability=True)
        olab, oprob = so.predict_probability(m, Kt[t])
        assert lab_p == olab
        assert np.allclose(prob, oprob, rtol=1e-12, atol=1e-14)
        assert abs(prob.sum() - 1.0) < 1e-12
        assert np.allclose(prob, clf.predict_proba(Kt[t:t + 1])[0], atol=0.01)


def test_c_svc_without_probability(tmp_path, data):
    K, Kt, _, y3, _ = data
    clf = sklearn_svm.SVC(kernel="precomputed", C=1.0).fit(K, y3)
    m = _model_of(clf, "c_svc", clf.classes_)
    so.write_model(tmp_path / "m", m)
    model = ska.SVMModel(tmp_path / "m")
    assert not model.has_probability
    for t in range(Kt.shape[0]):
        # SVMPredict asks for probabilities; svm_predict_probability falls
        # back to svm_predict's vote and the estimates stay zero
        lab, prob = model.predict(Kt[t], probability=True)
        assert lab == clf.predict(Kt[t:t + 1])[0] == so.predict(m, Kt[t])
        assert np.all(prob == 0.0)


def test_one_class_and_svr(tmp_path, data):
    K, Kt, _, _, yr = data
    oc = sklearn_svm.OneClassSVM(kernel="precomputed", nu=0.3).fit(K)
    m = _model_of(oc, "one_class")
    so.write_model(tmp_path / "oc", m)
    model = ska.SVMModel(tmp_path / "oc")
    for t in range(Kt.shape[0]):
        lab, dec = model.predict(Kt[t], probability=True)  # not a classifier: decision values
        assert np.allclose(dec[0], oc.decision_function(Kt[t:t + 1])[0], rtol=1e-10, atol=1e-12)
        assert lab == oc.predict(Kt[t:t + 1])[0]
    svr = sklearn_svm.SVR(kernel="precomputed", C=3.0, epsilon=0.05).fit(K, yr)
    m = _model_of(svr, "epsilon_svr")
    so.write_model(tmp_path / "svr", m)
    model = ska.SVMModel(tmp_path / "svr")
    for t in range(Kt.shape[0]):
        lab, dec = model.predict(Kt[t])
        assert np.isclose(lab, svr.predict(Kt[t:t + 1])[0], rtol=1e-10, atol=1e-12) and lab == dec[0]


def test_feature_kernels(tmp_path):
    """Non-precomputed models evaluate the kernel on the test vector (the
    kernel row as features, x[0] = the test's running count)."""
    row = np.array([0.5, -1.0, 2.0])
    svs = {1: 0.25, 3: -0.5}  # one SV: indices 1 and 3 of the feature vector
    x = {0: 7.0, 1: 0.5, 2: -1.0, 3: 2.0}
    dot = sum(v * x[i] for i, v in svs.items())
    sq = sum((x.get(i, 0.0) - svs.get(i, 0.0)) ** 2 for i in set(x) | set(svs))
    cases = {"linear": dot, "polynomial": (0.5 * dot + 1.0) ** 3, "rbf": np.exp(-0.5 * sq),
             "sigmoid": np.tanh(0.5 * dot + 1.0)}
    for kt, kval in cases.items():
        path = tmp_path / kt
        path.write_text(f"svm_type epsilon_svr\nkernel_type {kt}\ndegree 3\ngamma 0.5\ncoef0 1\n"
                        "nr_class 2\ntotal_sv 1\nrho 0.25\nSV\n2 1:0.25 3:-0.5 \n")
        lab, dec = ska.SVMModel(path).predict(row, cnt=7)
        assert np.isclose(dec[0], 2 * kval - 0.25, rtol=1e-14, atol=1e-15), kt


def test_model_errors(tmp_path):
    with pytest.raises(ska.StemKernelError, match="no such file"):
        ska.SVMModel(tmp_path / "missing")
    (tmp_path / "bad").write_text("svm_type c_svx\n")
    with pytest.raises(ska.StemKernelError, match="unknown svm type"):
        ska.SVMModel(tmp_path / "bad")
    (tmp_path / "unk").write_text("svm_type c_svc\nfoo 1\n")
    with pytest.raises(ska.StemKernelError, match="unknown text in model file"):
        ska.SVMModel(tmp_path / "unk")
    (tmp_path / "far").write_text("svm_type c_svc\nkernel_type precomputed\nnr_class 2\ntotal_sv 1\n"
                                  "rho 0\nlabel 1 -1\nnr_sv 1 0\nSV\n1 0:9 \n")
    with pytest.raises(ska.StemKernelError, match="outside the kernel row"):
        ska.SVMModel(tmp_path / "far").predict(np.ones(3))
