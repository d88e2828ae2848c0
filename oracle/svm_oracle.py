"""Test oracle (never imported by the product): pure-Python restatement of the
libsvm 2.8x prediction path the reference's SVMPredict uses for predict
mode's Output (libsvm/svm_util.cpp:41-95), for the precomputed kernel:

  svm_predict_values       libsvm/svm.cpp:1053-1106
  svm_predict              libsvm/svm.cpp:1108-1150
  svm_predict_probability  libsvm/svm.cpp:1152-1189
  sigmoid_predict          libsvm/svm.cpp:416-423
  multiclass_probability   libsvm/svm.cpp:426-488
  Kernel::k_function (PRECOMPUTED)  libsvm/qmatrix.cpp:296-297

A model is a dict: svm_type ("c_svc", ...), nr_class, label, nSV, rho,
probA, probB, sv_coef (list of nr_class-1 lists), sv_index (1-based training
indices of the SVs).  Pinned in tests/test_svm_predict.py against
scikit-learn's libsvm on the same models (labels and decision values)."""
import math


def decision_values(m, row):
    x = [0.0] + list(row)  # make_svm_node: x[i] holds row[i-1]; x[0] = cnt (unused here)
    kv = [x[int(i)] for i in m["sv_index"]]
    if m["svm_type"] in ("one_class", "epsilon_svr", "nu_svr"):
        return [sum(c * k for c, k in zip(m["sv_coef"][0], kv)) - m["rho"][0]]
    k = m["nr_class"]
    start = [0] * k
    for i in range(1, k):
        start[i] = start[i - 1] + m["nSV"][i - 1]
    dec = []
    p = 0
    for i in range(k):
        for j in range(i + 1, k):
            s = 0.0
            for t in range(m["nSV"][i]):
                s += m["sv_coef"][j - 1][start[i] + t] * kv[start[i] + t]
            for t in range(m["nSV"][j]):
                s += m["sv_coef"][i][start[j] + t] * kv[start[j] + t]
            dec.append(s - m["rho"][p])
            p += 1
    return dec


def predict(m, row):
    dec = decision_values(m, row)
    if m["svm_type"] == "one_class":
        return 1.0 if dec[0] > 0 else -1.0
    if m["svm_type"] in ("epsilon_svr", "nu_svr"):
        return dec[0]
    k = m["nr_class"]
    vote = [0] * k
    pos = 0
    for i in range(k):
        for j in range(i + 1, k):
            if dec[pos] > 0:
                vote[i] += 1
            else:
                vote[j] += 1
            pos += 1
    best = 0
    for i in range(1, k):
        if vote[i] > vote[best]:
            best = i
    return float(m["label"][best])


def sigmoid_predict(dv, A, B):
    f = dv * A + B
    if f >= 0:
        return math.exp(-f) / (1.0 + math.exp(-f))
    return 1.0 / (1 + math.exp(f))


def multiclass_probability(k, r):
    max_iter = max(100, k)
    eps = 0.005 / k
    p = [1.0 / k] * k
    Q = [[0.0] * k for _ in range(k)]
    for t in range(k):
        for j in range(t):
            Q[t][t] += r[j][t] * r[j][t]
            Q[t][j] = Q[j][t]
        for j in range(t + 1, k):
            Q[t][t] += r[j][t] * r[j][t]
            Q[t][j] = -r[j][t] * r[t][j]
    Qp = [0.0] * k
    for _ in range(max_iter):
        pQp = 0.0
        for t in range(k):
            Qp[t] = sum(Q[t][j] * p[j] for j in range(k))
            pQp += p[t] * Qp[t]
        if max(abs(Qp[t] - pQp) for t in range(k)) < eps:
            break
        for t in range(k):
            diff = (-Qp[t] + pQp) / Q[t][t]
            p[t] += diff
            pQp = (pQp + diff * (diff * Q[t][t] + 2 * Qp[t])) / (1 + diff) / (1 + diff)
            for j in range(k):
                Qp[j] = (Qp[j] + diff * Q[t][j]) / (1 + diff)
                p[j] /= (1 + diff)
    return p


def predict_probability(m, row):
    k = m["nr_class"]
    dec = decision_values(m, row)
    r = [[0.0] * k for _ in range(k)]
    p = 0
    for i in range(k):
        for j in range(i + 1, k):
            r[i][j] = min(max(sigmoid_predict(dec[p], m["probA"][p], m["probB"][p]), 1e-7), 1 - 1e-7)
            r[j][i] = 1 - r[i][j]
            p += 1
    prob = multiclass_probability(k, r)
    best = 0
    for i in range(1, k):
        if prob[i] > prob[best]:
            best = i
    return float(m["label"][best]), prob


def write_model(path, m):
    """libsvm's model text (the format svm_load_model reads)."""
    with open(path, "w") as f:
        f.write(f"svm_type {m['svm_type']}\nkernel_type precomputed\n")
        f.write(f"nr_class {m['nr_class']}\ntotal_sv {len(m['sv_index'])}\n")
        f.write("rho " + " ".join(repr(float(v)) for v in m["rho"]) + "\n")
        if m.get("label") is not None:
            f.write("label " + " ".join(str(int(v)) for v in m["label"]) + "\n")
        if m.get("probA") is not None:
            f.write("probA " + " ".join(repr(float(v)) for v in m["probA"]) + "\n")
            f.write("probB " + " ".join(repr(float(v)) for v in m["probB"]) + "\n")
        if m.get("nSV") is not None:
            f.write("nr_sv " + " ".join(str(int(v)) for v in m["nSV"]) + "\n")
        f.write("SV\n")
        for t, idx in enumerate(m["sv_index"]):
            f.write(" ".join(repr(float(c[t])) for c in m["sv_coef"]) + f" 0:{int(idx)} \n")
