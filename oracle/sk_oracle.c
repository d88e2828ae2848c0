/*
 * sk_oracle.c -- CPU ORACLE (test infrastructure only; see sk_oracle.h).
 *
 * Plain-C restatement of the reference stem_kernel_lite path:
 *   ProfileSequence            common/profile.cpp:9-89
 *   char2rna                   common/rna.cpp:173-231
 *   BPMatrix averaging         common/bpmatrix.cpp:292-342, 399-417
 *   Profiler                   stem_kernel_lite/data.cpp:33-132
 *   DAGBuilder                 stem_kernel_lite/data.cpp:141-307
 *   find_root/find_max_parent  stem_kernel_lite/data.cpp:396-435
 *   fill_weight                stem_kernel_lite/data.cpp:437-453
 *   StemKernel::operator()     stem_kernel_lite/stem_kernel.cpp:14-95
 *   Simple/SubstNodeScore      stem_kernel_lite/score_table.cpp:14-53, 297-380
 *   SimpleEdgeScore            stem_kernel_lite/score_table.cpp:56-101
 *   StringKernel (profile)     stem_kernel_lite/string_kernel.cpp:10-132
 *   StringKernel (naive)       string_kernel/string_kernel.cpp:11-50
 * Loop orders and float/double intermediates follow the reference so that the
 * oracle reproduces its rounding; build with -ffp-contract=off.
 */
#include "sk_oracle.h"

#include <assert.h>
#include <ctype.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../stem_kernel_amd/csrc/ribosum85_60.inc"

#define NONE 0xffffffffu
enum { N_RNA = 4, RNA_GAP = 4 };

/* ------------------------------------------------------------------ */
/* alphabet: common/rna.cpp:173-231 (lower-case table search, default GAP) */
static const char kCharTab[17] = {'a', 'c', 'g', 'u', 't', '-', 'r', 'y', 'm',
                                  'k', 's', 'w', 'b', 'd', 'h', 'v', 'n'};
static const unsigned char kRnaTab[17] = {0, 1, 2, 3, 3, 4, 5,  6,  7,
                                          8, 9, 10, 11, 12, 13, 14, 15};

int orc_char2rna(int c) {
  char r = (char)tolower(c);
  for (int i = 0; i != 17; ++i)
    if (r == kCharTab[i]) return kRnaTab[i];
  return RNA_GAP;
}

/* IUPAC weights: common/profile.cpp:9-29 */
static const float kIupac[16][4] = {
    {1.0f, 0.0f, 0.0f, 0.0f},          {0.0f, 1.0f, 0.0f, 0.0f},
    {0.0f, 0.0f, 1.0f, 0.0f},          {0.0f, 0.0f, 0.0f, 1.0f},
    {0.0f, 0.0f, 0.0f, 0.0f},          {1.0 / 2, 0.0f, 1.0 / 2, 0.0f},
    {0.0f, 1.0 / 2, 0.0f, 1.0 / 2},    {1.0 / 2, 1.0 / 2, 0.0f, 0.0f},
    {0.0f, 0.0f, 1.0 / 2, 1.0 / 2},    {0.0f, 1.0 / 2, 1.0 / 2, 0.0f},
    {1.0 / 2, 0.0f, 0.0f, 1.0 / 2},    {0.0f, 1.0 / 3, 1.0 / 3, 1.0 / 3},
    {1.0 / 3, 0.0f, 1.0 / 3, 1.0 / 3}, {1.0 / 3, 1.0 / 3, 0.0f, 1.0 / 3},
    {1.0 / 3, 1.0 / 3, 1.0 / 3, 0.0f}, {1.0 / 4, 1.0 / 4, 1.0 / 4, 1.0 / 4},
};

void orc_ribosum_tables(float *s16, float *p256) {
  memcpy(s16, SK_RIBOSUM_S, sizeof(SK_RIBOSUM_S));
  memcpy(p256, SK_RIBOSUM_P, sizeof(SK_RIBOSUM_P));
}

/* ProfileSequence::add_sequence(string, w=1) (profile.cpp:55-73) */
static void profile_add(float *prof5, int len, const char *s, float *n_seqs) {
  for (int i = 0; i != len; ++i) {
    int r = orc_char2rna((unsigned char)s[i]);
    if (r != RNA_GAP) {
      for (int j = 0; j != N_RNA; ++j) prof5[i * 5 + j] += kIupac[r][j] * 1.0f;
    } else {
      prof5[i * 5 + RNA_GAP] += 1.0f;
    }
  }
  *n_seqs += 1.0f;
}

/* ------------------------------------------------------------------ */
/* bp matrices: 1-based p(i,j), i<j, packed strict upper triangle */
typedef struct {
  const double *p;
  int n;
} bpmat;

static size_t tri_index(int n, int i, int j) { /* 0-based i<j */
  return (size_t)i * n - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1);
}
static double bpm_get(const bpmat *m, int i1, int j1) {
  assert(i1 < j1 && j1 <= m->n);
  return m->p[tri_index(m->n, i1 - 1, j1 - 1)];
}

/* ------------------------------------------------------------------ */
/* Profiler: stem_kernel_lite/data.cpp:33-132 */
typedef struct {
  const char *seq;
  int len;           /* aligned length (seq_.size()) */
  const bpmat *bpm;  /* per-row (gap-erased) or averaged matrix */
  float w;
  float *pr;  /* single-row profile [len][5] */
  uint32_t *idx;
  float *nbp;
} profiler;

static void profiler_init(profiler *P, const char *seq, int len,
                          const bpmat *bpm, float w) {
  P->seq = seq;
  P->len = len;
  P->bpm = bpm;
  P->w = w;
  P->pr = (float *)calloc((size_t)len * 5, sizeof(float));
  float ns = 0.0f;
  profile_add(P->pr, len, seq, &ns);
  P->idx = (uint32_t *)malloc(sizeof(uint32_t) * len);
  P->nbp = (float *)malloc(sizeof(float) * len);
  for (int i = 0; i != len; ++i) {
    P->idx[i] = NONE;
    P->nbp[i] = 1.0f;
  }
  /* make_idxmap (data.cpp:84-92): GAP is '-' for std::string */
  uint32_t j = 0;
  for (int i = 0; i != len; ++i)
    if (seq[i] != '-') P->idx[i] = j++;
  /* non_bp_profile (data.cpp:94-123) */
  if (bpm->n != len) {
    for (int i = 0; i != len; ++i) {
      if (P->idx[i] != NONE) {
        for (int k = 0; k != i; ++k)
          if (P->idx[k] != NONE)
            P->nbp[i] -= bpm_get(bpm, P->idx[k] + 1, P->idx[i] + 1);
        for (int k = i + 1; k != len; ++k)
          if (P->idx[k] != NONE)
            P->nbp[i] -= bpm_get(bpm, P->idx[i] + 1, P->idx[k] + 1);
        if (P->nbp[i] < 0.0) P->nbp[i] = 0.0f;
      }
    }
  } else {
    for (int i = 0; i != len; ++i) {
      if (P->idx[i] != NONE) {
        for (int k = 0; k != i; ++k)
          if (P->idx[k] != NONE) P->nbp[i] -= bpm_get(bpm, k + 1, i + 1);
        for (int k = i + 1; k != len; ++k)
          if (P->idx[k] != NONE) P->nbp[i] -= bpm_get(bpm, i + 1, k + 1);
        if (P->nbp[i] < 0.0) P->nbp[i] = 0.0f;
      }
    }
  }
}

static void profiler_free(profiler *P) {
  free(P->pr);
  free(P->idx);
  free(P->nbp);
}

static float profiler_loop(const profiler *P, int i) {
  assert(P->idx[i] != NONE);
  return P->w * P->nbp[i];
}

/* std::map<bp_t,float> restated as a 16-slot ordered table (keys (a,b) with
 * a,b<4 iterate in the same lexicographic order as the std::map). */
typedef struct {
  int present[16];
  float val[16];
} bpmap;

static void profiler_bp(const profiler *P, int i, int j, bpmap *v) {
  if (P->idx[i] != NONE && P->idx[j] != NONE) {
    float p = (float)(P->bpm->n != P->len
                          ? bpm_get(P->bpm, P->idx[i] + 1, P->idx[j] + 1)
                          : bpm_get(P->bpm, i + 1, j + 1));
    for (int a = 0; a != N_RNA; ++a) {
      if (P->pr[i * 5 + a] == 0.0) continue;
      for (int b = 0; b != N_RNA; ++b) {
        if (P->pr[j * 5 + b] == 0.0) continue;
        int k = a * 4 + b;
        float add = P->w * p * P->pr[i * 5 + a] * P->pr[j * 5 + b];
        if (!v->present[k]) {
          v->present[k] = 1;
          v->val[k] = add;
        } else {
          v->val[k] += add;
        }
      }
    }
  }
}

/* ------------------------------------------------------------------ */
/* DAG storage: stem_kernel_lite/dag.h:17-157 */
typedef struct {
  uint32_t to, gaps;
} oedge;
typedef struct {
  uint32_t code;
  float p;
} obpf;
typedef struct {
  uint32_t first, last;
  float weight;
  oedge *edges;
  int n_edges;
  obpf *bpf;
  int n_bpf;
} onode;

struct orc_mdata {
  int len;      /* aligned length */
  int n_rows;
  onode *tree;
  int n_nodes, cap_nodes;
  uint32_t *root;
  int n_root;
  uint32_t *max_pa;
  float *weight; /* per position; NULL if !use_bp */
  float *prof5;  /* ProfileSequence of all rows [len][5] */
  float n_seqs;
  double *bpp;   /* averaged matrix, packed over len (NULL if !use_bp) */
};

/* growable Pos list (std::list<Pos> in the reference) */
typedef struct {
  uint32_t *a, *b;
  int n, cap;
} plist;

static void plist_push(plist *l, uint32_t a, uint32_t b) {
  if (l->n == l->cap) {
    l->cap = l->cap ? l->cap * 2 : 4;
    l->a = (uint32_t *)realloc(l->a, sizeof(uint32_t) * l->cap);
    l->b = (uint32_t *)realloc(l->b, sizeof(uint32_t) * l->cap);
  }
  l->a[l->n] = a;
  l->b[l->n] = b;
  l->n++;
}
static void plist_free(plist *l) {
  free(l->a);
  free(l->b);
  l->a = l->b = NULL;
  l->n = l->cap = 0;
}

/* CYKTable cell (i<=j) index for a size-sz table */
static size_t cyk(int i, int j) { return (size_t)j * (j + 1) / 2 + (size_t)i; }

typedef struct {
  const profiler *prof;
  int n_prof;
  const bpmat *bpm;
  float th;
  int sz;
  plist *bp;    /* CYKTable<list<Pos>> bp_ */
  plist *head;  /* vector<list<Pos>> head_ */
  uint32_t *vt; /* CYKTable<uint> vt_ */
  orc_mdata *d;
} dagbuilder;

/* DAGBuilder::initialize (data.cpp:165-191) */
static void dag_initialize(dagbuilder *B) {
  int sz = B->sz;
  size_t ncell = (size_t)sz * (sz + 1) / 2;
  plist *ch = (plist *)calloc(ncell ? ncell : 1, sizeof(plist));
  for (int j = 1; j < sz; ++j) {
    for (int i = j - 1;; --i) {
      if (bpm_get(B->bpm, i + 1, j + 1) >= (double)B->th) {
        /* std::swap(bp_(i,j), ch(i+1,j-1)); bp_(i,j) is empty here, so this
         * moves the candidate list.  For j==i+1 the reference's CYKTable read
         * of (i+1,j-1) aliases a still-empty cell: the list is empty. */
        if (i + 1 <= j - 1) {
          plist t = B->bp[cyk(i, j)];
          B->bp[cyk(i, j)] = ch[cyk(i + 1, j - 1)];
          ch[cyk(i + 1, j - 1)] = t;
        }
        plist_push(&ch[cyk(i, j)], (uint32_t)i, (uint32_t)j);
        plist_push(&B->head[i], (uint32_t)i, (uint32_t)j);
      } else {
        /* remove_copy_if(ch(i+1,j), bind1st(is_child(), head_[i].back()))
         * then copy head_[i].  head_[i].back() on an empty libstdc++ list
         * reads the node header's size word: Pos(0,0) (SURVEY App.A #2). */
        uint32_t hb = B->head[i].n ? B->head[i].b[B->head[i].n - 1] : 0u;
        plist *src = &ch[cyk(i + 1, j)];
        plist *dst = &ch[cyk(i, j)];
        for (int k = 0; k != src->n; ++k)
          if (!(hb > src->b[k])) plist_push(dst, src->a[k], src->b[k]);
        for (int k = 0; k != B->head[i].n; ++k)
          plist_push(dst, B->head[i].a[k], B->head[i].b[k]);
      }
      if (i == 0) break;
    }
  }
  for (size_t c = 0; c != ncell; ++c) plist_free(&ch[c]);
  free(ch);
  for (size_t c = 0; c != ncell; ++c) B->vt[c] = NONE;
}

static float dag_loop_profile(const dagbuilder *B, int i) {
  float v = 0.0f, t = 0.0f;
  for (int p = 0; p != B->n_prof; ++p) {
    if (B->prof[p].idx[i] != NONE) v += profiler_loop(&B->prof[p], i);
    t += B->prof[p].w;
  }
  return v / t;
}

static void dag_bp_profile(const dagbuilder *B, int i, int j, onode *nd) {
  bpmap v;
  memset(&v, 0, sizeof(v));
  float t = 0.0f;
  for (int p = 0; p != B->n_prof; ++p) {
    if (B->prof[p].idx[i] != NONE && B->prof[p].idx[j] != NONE)
      profiler_bp(&B->prof[p], i, j, &v);
    t += B->prof[p].w;
  }
  int n = 0;
  for (int k = 0; k != 16; ++k) n += v.present[k];
  nd->bpf = (obpf *)malloc(sizeof(obpf) * (n ? n : 1));
  nd->n_bpf = 0;
  for (int k = 0; k != 16; ++k)
    if (v.present[k]) {
      nd->bpf[nd->n_bpf].code = (uint32_t)k;
      nd->bpf[nd->n_bpf].p = v.val[k] / t;
      nd->n_bpf++;
    }
}

static uint32_t tree_push(orc_mdata *d, const onode *n) {
  if (d->n_nodes == d->cap_nodes) {
    d->cap_nodes = d->cap_nodes ? d->cap_nodes * 2 : 64;
    d->tree = (onode *)realloc(d->tree, sizeof(onode) * d->cap_nodes);
  }
  d->tree[d->n_nodes] = *n;
  return (uint32_t)d->n_nodes++;
}

static uint32_t dag_build_helper(dagbuilder *B, uint32_t a, uint32_t b);

/* make_loop (data.cpp:200-211) */
static void dag_make_loop(dagbuilder *B, uint32_t a, uint32_t b) {
  onode nd;
  memset(&nd, 0, sizeof(nd));
  nd.first = a;
  nd.last = b;
  dag_bp_profile(B, (int)a, (int)b, &nd);
  nd.weight = dag_loop_profile(B, (int)a) * dag_loop_profile(B, (int)b);
  uint32_t ret = dag_build_helper(B, a, a);
  nd.edges = (oedge *)malloc(sizeof(oedge));
  nd.n_edges = 1;
  nd.edges[0].to = ret;
  nd.edges[0].gaps = b - a - 1; /* Edge(to, p_pos): dag.h:29-33 */
  B->vt[cyk((int)a, (int)b)] = tree_push(B->d, &nd);
}

/* make_stem (data.cpp:213-229) */
static void dag_make_stem(dagbuilder *B, uint32_t a, uint32_t b) {
  const plist cur = B->bp[cyk((int)a, (int)b)];
  onode nd;
  memset(&nd, 0, sizeof(nd));
  nd.first = a;
  nd.last = b;
  dag_bp_profile(B, (int)a, (int)b, &nd);
  nd.weight = dag_loop_profile(B, (int)a) * dag_loop_profile(B, (int)b);
  nd.edges = (oedge *)malloc(sizeof(oedge) * cur.n);
  nd.n_edges = cur.n;
  for (int k = 0; k != cur.n; ++k) {
    uint32_t ret = dag_build_helper(B, cur.a[k], cur.b[k]);
    nd.edges[k].to = ret;
    /* Edge(to, p_pos, c_pos): dag.h:22-27 */
    nd.edges[k].gaps = (cur.a[k] - a - 1) + (b - cur.b[k] - 1);
  }
  B->vt[cyk((int)a, (int)b)] = tree_push(B->d, &nd);
}

/* build_helper (data.cpp:231-244) */
static uint32_t dag_build_helper(dagbuilder *B, uint32_t a, uint32_t b) {
  if (B->vt[cyk((int)a, (int)b)] == NONE) {
    if (a == b) {
      onode leaf;
      memset(&leaf, 0, sizeof(leaf));
      leaf.first = a;
      leaf.last = b;
      leaf.weight = 1.0f;
      B->vt[cyk((int)a, (int)b)] = tree_push(B->d, &leaf);
    } else if (B->bp[cyk((int)a, (int)b)].n == 0) {
      dag_make_loop(B, a, b);
    } else {
      dag_make_stem(B, a, b);
    }
  }
  return B->vt[cyk((int)a, (int)b)];
}

/* ------------------------------------------------------------------ */
orc_mdata *orc_mdata_new(int n_rows, const char *const *rows,
                         const double *const *bpp_rows, float th, int use_bp) {
  orc_mdata *d = (orc_mdata *)calloc(1, sizeof(orc_mdata));
  int L = (int)strlen(rows[0]);
  d->len = L;
  d->n_rows = n_rows;
  for (int r = 0; r != n_rows; ++r) assert((int)strlen(rows[r]) == L);
  d->prof5 = (float *)calloc((size_t)L * 5, sizeof(float));
  d->n_seqs = 0.0f;
  for (int r = 0; r != n_rows; ++r) profile_add(d->prof5, L, rows[r], &d->n_seqs);
  if (!use_bp) return d;

  /* BPMatrix(list<string>) FOLD path: per-row fold of erase_gap(lowercase(row))
   * then average_matrix (bpmatrix.cpp:306-342, 399-417). */
  size_t npk = L > 1 ? (size_t)L * (L - 1) / 2 : 1;
  d->bpp = (double *)calloc(npk, sizeof(double));
  bpmat *rowm = (bpmat *)malloc(sizeof(bpmat) * n_rows);
  for (int r = 0; r != n_rows; ++r) {
    int *idxmap = (int *)malloc(sizeof(int) * L);
    int nr = 0;
    for (int i = 0; i != L; ++i) idxmap[i] = (rows[r][i] != '-') ? nr++ : -1;
    rowm[r].p = bpp_rows[r];
    rowm[r].n = nr;
    for (int j = 1; j < L; ++j) {
      if (idxmap[j] < 0) continue;
      for (int i = j - 1;; --i) {
        if (idxmap[i] >= 0)
          d->bpp[tri_index(L, i, j)] += bpm_get(&rowm[r], idxmap[i] + 1, idxmap[j] + 1);
        if (i == 0) break;
      }
    }
    free(idxmap);
  }
  for (size_t k = 0; k != npk; ++k) d->bpp[k] = d->bpp[k] / n_rows;
  bpmat avg = {d->bpp, L};

  /* MData ctor: per-row matrices when n_matrices()>1, else the averaged one */
  profiler *prof = (profiler *)malloc(sizeof(profiler) * n_rows);
  for (int r = 0; r != n_rows; ++r)
    profiler_init(&prof[r], rows[r], L, n_rows > 1 ? &rowm[r] : &avg, 1.0f);

  dagbuilder B;
  memset(&B, 0, sizeof(B));
  B.prof = prof;
  B.n_prof = n_rows;
  B.bpm = &avg;
  B.th = th;
  B.sz = L;
  size_t ncell = (size_t)L * (L + 1) / 2;
  B.bp = (plist *)calloc(ncell ? ncell : 1, sizeof(plist));
  B.head = (plist *)calloc(L ? L : 1, sizeof(plist));
  B.vt = (uint32_t *)malloc(sizeof(uint32_t) * (ncell ? ncell : 1));
  B.d = d;
  dag_initialize(&B);
  /* build (data.cpp:151-160): heads of each i in reverse push order */
  for (int i = 0; i != L; ++i)
    for (int k = B.head[i].n - 1; k >= 0; --k)
      dag_build_helper(&B, B.head[i].a[k], B.head[i].b[k]);

  /* find_root (data.cpp:396-418) */
  char *is_root = (char *)malloc(d->n_nodes ? d->n_nodes : 1);
  memset(is_root, 1, d->n_nodes);
  for (int i = 0; i != d->n_nodes; ++i)
    for (int e = 0; e != d->tree[i].n_edges; ++e) is_root[d->tree[i].edges[e].to] = 0;
  d->n_root = 0;
  for (int i = 0; i != d->n_nodes; ++i) d->n_root += is_root[i];
  d->root = (uint32_t *)malloc(sizeof(uint32_t) * (d->n_root ? d->n_root : 1));
  int c = 0;
  for (int i = 0; i != d->n_nodes; ++i)
    if (is_root[i]) d->root[c++] = (uint32_t)i;
  free(is_root);
  /* find_max_parent (data.cpp:420-435) */
  d->max_pa = (uint32_t *)malloc(sizeof(uint32_t) * (d->n_nodes ? d->n_nodes : 1));
  for (int i = 0; i != d->n_nodes; ++i) d->max_pa[i] = NONE;
  for (int i = 0; i != d->n_nodes; ++i)
    for (int e = 0; e != d->tree[i].n_edges; ++e) {
      uint32_t t = d->tree[i].edges[e].to;
      if (d->max_pa[t] == NONE || d->max_pa[t] < (uint32_t)i) d->max_pa[t] = (uint32_t)i;
    }
  /* fill_weight (data.cpp:437-453) */
  d->weight = (float *)malloc(sizeof(float) * (L ? L : 1));
  for (int i = 0; i != L; ++i) {
    float v = 0.0f, t = 0.0f;
    for (int p = 0; p != n_rows; ++p) {
      if (prof[p].idx[i] != NONE) v += profiler_loop(&prof[p], i);
      t += prof[p].w;
    }
    d->weight[i] = v / t;
  }

  for (size_t k = 0; k != ncell; ++k) plist_free(&B.bp[k]);
  for (int i = 0; i != L; ++i) plist_free(&B.head[i]);
  free(B.bp);
  free(B.head);
  free(B.vt);
  for (int r = 0; r != n_rows; ++r) profiler_free(&prof[r]);
  free(prof);
  free(rowm);
  return d;
}

void orc_mdata_free(orc_mdata *d) {
  if (!d) return;
  for (int i = 0; i != d->n_nodes; ++i) {
    free(d->tree[i].edges);
    free(d->tree[i].bpf);
  }
  free(d->tree);
  free(d->root);
  free(d->max_pa);
  free(d->weight);
  free(d->prof5);
  free(d->bpp);
  free(d);
}

int orc_mdata_n_nodes(const orc_mdata *d) { return d->n_nodes; }
int orc_mdata_seq_len(const orc_mdata *d) { return d->len; }
int orc_mdata_n_edges(const orc_mdata *d) {
  int n = 0;
  for (int i = 0; i != d->n_nodes; ++i) n += d->tree[i].n_edges;
  return n;
}
int orc_mdata_n_bpfreq(const orc_mdata *d) {
  int n = 0;
  for (int i = 0; i != d->n_nodes; ++i) n += d->tree[i].n_bpf;
  return n;
}
void orc_mdata_nodes(const orc_mdata *d, uint32_t *first, uint32_t *last,
                     uint32_t *n_edges, uint32_t *n_bpfreq, float *weight,
                     uint32_t *max_pa) {
  for (int i = 0; i != d->n_nodes; ++i) {
    first[i] = d->tree[i].first;
    last[i] = d->tree[i].last;
    n_edges[i] = (uint32_t)d->tree[i].n_edges;
    n_bpfreq[i] = (uint32_t)d->tree[i].n_bpf;
    weight[i] = d->tree[i].weight;
    max_pa[i] = d->max_pa[i];
  }
}
void orc_mdata_edges(const orc_mdata *d, uint32_t *to, uint32_t *gaps) {
  int k = 0;
  for (int i = 0; i != d->n_nodes; ++i)
    for (int e = 0; e != d->tree[i].n_edges; ++e, ++k) {
      to[k] = d->tree[i].edges[e].to;
      gaps[k] = d->tree[i].edges[e].gaps;
    }
}
void orc_mdata_bpfreq(const orc_mdata *d, uint32_t *code, float *p) {
  int k = 0;
  for (int i = 0; i != d->n_nodes; ++i)
    for (int e = 0; e != d->tree[i].n_bpf; ++e, ++k) {
      code[k] = d->tree[i].bpf[e].code;
      p[k] = d->tree[i].bpf[e].p;
    }
}
int orc_mdata_n_roots(const orc_mdata *d) { return d->n_root; }
void orc_mdata_roots(const orc_mdata *d, uint32_t *roots) {
  memcpy(roots, d->root, sizeof(uint32_t) * d->n_root);
}
void orc_mdata_weight(const orc_mdata *d, float *w) {
  if (d->weight) memcpy(w, d->weight, sizeof(float) * d->len);
}
void orc_mdata_profile(const orc_mdata *d, float *prof5, float *n_seqs) {
  memcpy(prof5, d->prof5, sizeof(float) * 5 * d->len);
  *n_seqs = d->n_seqs;
}
void orc_mdata_bpp(const orc_mdata *d, double *packed) {
  if (d->bpp && d->len > 1)
    memcpy(packed, d->bpp, sizeof(double) * (size_t)d->len * (d->len - 1) / 2);
}

/* ------------------------------------------------------------------ */
/* StemKernel<ST,MData>::operator() (stem_kernel_lite/stem_kernel.cpp:14-95)
 * with SubstScoreTable (subst=1) or SimpleScoreTable (subst=0). */
typedef struct {
  int subst;
  double gap; /* loop_gap: SimpleEdgeScore gap_ and node gap_ */
  double co_subst[256];
  double match, mismatch;
  unsigned band;
} stem_params;

static double *gap_powers(double gap, int n) {
  /* SimpleEdgeScore::initialize (score_table.cpp:60-77): g[k]=g[k-1]*gap */
  double *g = (double *)malloc(sizeof(double) * (n > 1 ? n : 1));
  g[0] = 1.0;
  for (int k = 1; k < n; ++k) g[k] = g[k - 1] * gap;
  return g;
}

static double node_gap_score(const stem_params *S, const orc_mdata *d, int i) {
  return S->gap * S->gap * d->tree[i].weight; /* score_table.h:26-29, 51-54 */
}

static double node_match_score(const stem_params *S, const orc_mdata *x,
                               const orc_mdata *y, int i, int j) {
  const onode *ni = &x->tree[i], *nj = &y->tree[j];
  double v_c = 0.0;
  for (int a = 0; a != ni->n_bpf; ++a) {
    double cx = ni->bpf[a].p;
    for (int b = 0; b != nj->n_bpf; ++b) {
      double cy = nj->bpf[b].p;
      double v;
      if (S->subst) {
        v = S->co_subst[ni->bpf[a].code * 16 + nj->bpf[b].code];
      } else {
        v = (ni->bpf[a].code != nj->bpf[b].code) ? S->mismatch : S->match;
      }
      v_c += v * cx * cy;
    }
  }
  double nbp_x = x->prof5[ni->first * 5 + RNA_GAP];
  v_c += node_gap_score(S, y, j) * nbp_x / (double)x->n_seqs;
  double nbp_y = y->prof5[nj->first * 5 + RNA_GAP];
  v_c += node_gap_score(S, x, i) * nbp_y / (double)y->n_seqs;
  return v_c;
}

static double stem_dp(const stem_params *S, const orc_mdata *x, const orc_mdata *y) {
  int nx = x->n_nodes, ny = y->n_nodes;
  int glen = 2 * (x->len > y->len ? x->len : y->len);
  double *g = gap_powers(S->gap, glen + 2);
  size_t cells = (size_t)(nx ? nx : 1) * (ny ? ny : 1);
  double *K0 = (double *)malloc(sizeof(double) * cells);
  double *G0 = (double *)malloc(sizeof(double) * cells);
  double *K1 = (double *)calloc(ny ? ny : 1, sizeof(double));
  double *G1 = (double *)calloc(ny ? ny : 1, sizeof(double));
#define AT(M, a, b) M[(size_t)(a) * ny + (b)]
  for (int i = 0; i != nx; ++i) {
    const onode *xi = &x->tree[i];
    for (int j = 0; j != ny; ++j) {
      const onode *yj = &y->tree[j];
      if (xi->n_edges == 0 && yj->n_edges == 0) {
        AT(K0, i, j) = AT(G0, i, j) = 1.0;
        continue;
      }
      K1[j] = G1[j] = 0.0;
      if (xi->n_edges && yj->n_edges &&
          (S->band == 0 ||
           (unsigned)abs((int)((xi->last - xi->first) - (yj->last - yj->first))) <= S->band)) {
        double v_s = node_match_score(S, x, y, i, j);
        for (int ex = 0; ex != xi->n_edges; ++ex) {
          for (int ey = 0; ey != yj->n_edges; ++ey) {
            double e_s = g[xi->edges[ex].gaps] * g[yj->edges[ey].gaps] * 1.0f * 1.0f;
            double v = AT(G0, xi->edges[ex].to, yj->edges[ey].to) * v_s * e_s;
            K1[j] += v;
            G1[j] += v;
          }
        }
      }
      for (int ey = 0; ey != yj->n_edges; ++ey) {
        double v_s = node_gap_score(S, y, j);
        double e_s = g[yj->edges[ey].gaps] * 1.0f;
        K1[j] += K1[yj->edges[ey].to];
        G1[j] += G1[yj->edges[ey].to] * v_s * e_s;
      }
      AT(K0, i, j) = K1[j];
      AT(G0, i, j) = G1[j];
      for (int ex = 0; ex != xi->n_edges; ++ex) {
        double v_s = node_gap_score(S, x, i);
        double e_s = g[xi->edges[ex].gaps] * 1.0f;
        AT(K0, i, j) += AT(K0, xi->edges[ex].to, j);
        AT(G0, i, j) += AT(G0, xi->edges[ex].to, j) * v_s * e_s;
      }
    }
  }
  double ret = 0.0;
  for (int a = 0; a != x->n_root; ++a)
    for (int b = 0; b != y->n_root; ++b) ret += AT(K0, x->root[a], y->root[b]);
#undef AT
  free(K0);
  free(G0);
  free(K1);
  free(G1);
  free(g);
  return ret;
}

double orc_su_stem(const orc_mdata *x, const orc_mdata *y, double loop_gap,
                   double beta, unsigned band) {
  stem_params S;
  memset(&S, 0, sizeof(S));
  S.subst = 1;
  S.gap = loop_gap;
  S.band = band;
  /* SubstNodeScore ctor (score_table.cpp:118-134) */
  for (int k = 0; k != 256; ++k) S.co_subst[k] = exp(SK_RIBOSUM_P[k] * beta);
  return stem_dp(&S, x, y);
}

double orc_si_stem(const orc_mdata *x, const orc_mdata *y, double loop_gap,
                   double stack, double covar, unsigned band) {
  stem_params S;
  memset(&S, 0, sizeof(S));
  S.subst = 0;
  S.gap = loop_gap;
  S.match = stack;
  S.mismatch = covar;
  S.band = band;
  return stem_dp(&S, x, y);
}

/* ------------------------------------------------------------------ */
/* StringKernel<double,MData> (stem_kernel_lite/string_kernel.cpp) */
static double prof_subst(const double *st, const float *x, const float *y) {
  double v_c = 0.0;
  float n = 0;
  for (int i = 0; i != N_RNA; ++i) {
    if (x[i] == 0) continue;
    for (int j = 0; j != N_RNA; ++j) {
      if (y[j] == 0) continue;
      n += x[i] * y[j];
      v_c += st[i * 4 + j] * x[i] * y[j];
    }
  }
  return n == 0 ? 1.0 : v_c / n;
}

double orc_profile_string(const orc_mdata *xx, const orc_mdata *yy, double gap,
                          int ribosum, double alpha, double match,
                          double mismatch) {
  double st[16];
  for (int i = 0; i != 4; ++i)
    for (int k = 0; k != 4; ++k)
      st[i * 4 + k] = ribosum ? exp(SK_RIBOSUM_S[i * 4 + k] * alpha)
                              : (i == k ? match : mismatch);
  int sx = xx->len, sy = yy->len;
  int use_weight = xx->weight != NULL && yy->weight != NULL && sx > 0 && sy > 0;
  double *K0p = (double *)malloc(sizeof(double) * (sy + 1));
  double *G0p = (double *)malloc(sizeof(double) * (sy + 1));
  double *K0c = (double *)malloc(sizeof(double) * (sy + 1));
  double *G0c = (double *)malloc(sizeof(double) * (sy + 1));
  double *K1 = (double *)calloc(sy + 1, sizeof(double));
  double *G1 = (double *)calloc(sy + 1, sizeof(double));
  K0p[0] = G0p[0] = 1.0;
  for (int j = 1; j != sy + 1; ++j) {
    K0p[j] = 1.0;
    G0p[j] = G0p[j - 1] * gap;
  }
  for (int i = 1; i != sx + 1; ++i) {
    K0c[0] = 1.0;
    G0c[0] = G0p[0] * gap;
    K1[0] = G1[0] = 0.0;
    for (int j = 1; j != sy + 1; ++j) {
      double v;
      if (use_weight) {
        v = G0p[j - 1] * xx->weight[i - 1] * yy->weight[j - 1];
      } else {
        v = G0p[j - 1];
      }
      v *= prof_subst(st, &xx->prof5[(i - 1) * 5], &yy->prof5[(j - 1) * 5]);
      K1[j] = v + K1[j - 1];
      G1[j] = v + G1[j - 1] * gap;
      K0c[j] = K1[j] + K0p[j];
      G0c[j] = G1[j] + G0p[j] * gap;
    }
    double *t;
    t = K0p; K0p = K0c; K0c = t;
    t = G0p; G0p = G0c; G0c = t;
  }
  double ret = K0p[sy];
  free(K0p); free(G0p); free(K0c); free(G0c); free(K1); free(G1);
  return ret;
}

/* ------------------------------------------------------------------ */
/* StringKernel<double>::operator() (string_kernel/string_kernel.cpp:11-50) */
double orc_naive_string(const char *x, const char *y, double gap) {
  int nx = (int)strlen(x), ny = (int)strlen(y);
  double g = gap, g2 = g * g;
  double *K0 = (double *)malloc(sizeof(double) * (size_t)(nx + 1) * (ny + 1));
  double *G0 = (double *)malloc(sizeof(double) * (size_t)(nx + 1) * (ny + 1));
  double *K1 = (double *)calloc(ny + 1, sizeof(double));
  double *G1 = (double *)calloc(ny + 1, sizeof(double));
#define A(M, i, j) M[(size_t)(i) * (ny + 1) + (j)]
  A(K0, 0, 0) = A(G0, 0, 0) = 1.0;
  for (int i = 1; i != nx + 1; ++i) {
    A(K0, i, 0) = 1.0;
    A(G0, i, 0) = A(G0, i - 1, 0) * g;
  }
  for (int j = 1; j != ny + 1; ++j) {
    A(K0, 0, j) = 1.0;
    A(G0, 0, j) = A(G0, 0, j - 1) * g;
  }
  for (int i = 1; i != nx + 1; ++i) {
    K1[0] = G1[0] = 0.0;
    for (int j = 1; j != ny + 1; ++j) {
      K1[j] = K1[j - 1];
      G1[j] = G1[j - 1] * g;
      if (x[i - 1] == y[j - 1]) {
        K1[j] += A(G0, i - 1, j - 1) * g2;
        G1[j] += A(G0, i - 1, j - 1) * g2;
      }
      A(K0, i, j) = A(K0, i - 1, j) + K1[j];
      A(G0, i, j) = A(G0, i - 1, j) * g + G1[j];
    }
  }
  double r = A(K0, nx, ny);
#undef A
  free(K0); free(G0); free(K1); free(G1);
  return r;
}

/* ------------------------------------------------------------------ */
/* BPLA kernel (bpla_kernel/).  Data<ProfileSequence, list<string>>:
 * profile of all rows + fill_weight over the averaged BPMatrix
 * (bpla_kernel/data.cpp:19-45). */
void orc_bpla_weights(const orc_mdata *d, float *p_left, float *p_right, float *p_unpair) {
  const int L = d->len;
  for (int i = 0; i < L; ++i) {
    float pl = 0.0f, pr = 0.0f, pu;
    /* p_r[i] += bp(j+1,i+1), j<i ; p_l[i] += bp(i+1,j+1), j>i: float
     * accumulators, each add done in double then stored (data.cpp:33-36) */
    for (int j = 0; j < i; ++j) pr = (float)((double)pr + d->bpp[tri_index(L, j, i)]);
    for (int j = i + 1; j < L; ++j) pl = (float)((double)pl + d->bpp[tri_index(L, i, j)]);
    pu = (float)(1.0 - (double)(pl + pr));           /* data.cpp:37 */
    if (pu < 0.0f) pu = 0.0f;                        /* data.cpp:38 */
    p_right[i] = (float)sqrt((double)pr);            /* data.cpp:39-41 */
    p_left[i] = (float)sqrt((double)pl);
    p_unpair[i] = (float)sqrt((double)pu);
  }
}

typedef struct {
  const orc_mdata *x, *y;
  const float *xl, *xr, *xu, *yl, *yr, *yu;
  const double *table; /* 4x4 */
  double alpha;
  int bp;              /* BPLAScore (1) or LAScore (0) */
} la_score;

/* LAScore::operator() (bpla_kernel.cpp:24-43): counts-weighted mean of the
 * score table over the residue columns, 0 when either column has none. */
static double la_score_fn(const la_score *S, int i, int j) {
  const float *xc = S->x->prof5 + (size_t)i * 5, *yc = S->y->prof5 + (size_t)j * 5;
  double v = 0.0;
  float n = 0.0f;
  for (int k = 0; k != 4; ++k) {
    if (xc[k] == 0.0f) continue;
    for (int l = 0; l != 4; ++l) {
      if (yc[l] == 0.0f) continue;
      n += xc[k] * yc[l];
      v += S->table[k * 4 + l] * xc[k] * yc[l];
    }
  }
  return n == 0.0f ? 0.0 : v / n;
}

/* BPLAScore::operator() (bpla_kernel.cpp:48-62); float products as written */
static double score_fn(const la_score *S, int i, int j) {
  if (!S->bp) return la_score_fn(S, i, j);
  float lr = S->xr[i] * S->yr[j];
  float ll = S->xl[i] * S->yl[j];
  float u = S->xu[i] * S->yu[j];
  return S->alpha * (double)(lr + ll) + (double)u * la_score_fn(S, i, j);
}

static double bpla_exp(const la_score *S, double beta, double gap, double ext) {
  /* local_alignment_exp (bpla_kernel.cpp:64-115) */
  const int n = S->x->len, m = S->y->len, W = m + 1;
  const double bg = exp(beta * gap), be = exp(beta * ext);
  size_t cells = (size_t)(n + 1) * (m + 1);
  double *M = (double *)calloc(cells, sizeof(double)), *X = (double *)calloc(cells, sizeof(double));
  double *Y = (double *)calloc(cells, sizeof(double)), *X2 = (double *)calloc(cells, sizeof(double));
  double *Y2 = (double *)calloc(cells, sizeof(double));
#define AT(T, i, j) T[(size_t)(i) * W + (j)]
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      AT(M, i, j) = exp(beta * score_fn(S, i - 1, j - 1)) *
                    (1 + AT(X, i - 1, j - 1) + AT(Y, i - 1, j - 1) + AT(M, i - 1, j - 1));
      AT(X, i, j) = bg * AT(M, i - 1, j) + be * AT(X, i - 1, j);
      AT(Y, i, j) = bg * (AT(M, i, j - 1) + AT(X, i, j - 1)) + be * AT(Y, i, j - 1);
      AT(X2, i, j) = AT(M, i - 1, j) + AT(X2, i - 1, j);
      AT(Y2, i, j) = AT(M, i, j - 1) + AT(X2, i, j - 1) + AT(Y2, i, j - 1);
    }
  double r = 1 + AT(X2, n, m) + AT(Y2, n, m) + AT(M, n, m);
#undef AT
  free(M); free(X); free(Y); free(X2); free(Y2);
  return r;
}

static double dmax(double a, double b) { return a < b ? b : a; }

static double bpla_max(const la_score *S, double gap, double ext) {
  /* local_alignment_max (bpla_kernel.cpp:117-157) */
  const int n = S->x->len, m = S->y->len, W = m + 1;
  size_t cells = (size_t)(n + 1) * (m + 1);
  double *M = (double *)calloc(cells, sizeof(double)), *X = (double *)calloc(cells, sizeof(double));
  double *Y = (double *)calloc(cells, sizeof(double));
  double Mmax = 0;
#define AT(T, i, j) T[(size_t)(i) * W + (j)]
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      double v = dmax(0.0, AT(M, i - 1, j - 1));
      v = dmax(v, AT(X, i - 1, j - 1));
      v = dmax(v, AT(Y, i - 1, j - 1));
      AT(M, i, j) = v + score_fn(S, i - 1, j - 1);
      Mmax = dmax(Mmax, AT(M, i, j));
      AT(X, i, j) = dmax(AT(M, i - 1, j) + gap, AT(X, i - 1, j) + ext);
      AT(Y, i, j) = dmax(dmax(AT(M, i, j - 1) + gap, AT(X, i, j - 1) + gap), AT(Y, i, j - 1) + ext);
    }
#undef AT
  free(M); free(X); free(Y);
  return Mmax;
}

double orc_bpla(const orc_mdata *x, const orc_mdata *y, int no_bp, int sw, double gap, double ext,
                double alpha, double beta, const double *table16) {
  /* BPLAKernel::operator() (bpla_kernel.cpp:159-174) */
  la_score S;
  memset(&S, 0, sizeof(S));
  S.x = x;
  S.y = y;
  S.table = table16;
  S.alpha = alpha;
  S.bp = !no_bp;
  float *w = NULL;
  if (S.bp) {
    if (!x->bpp || !y->bpp) return NAN; /* the reference indexes empty vectors */
    w = (float *)malloc(sizeof(float) * 3 * (size_t)(x->len + y->len + 1));
    float *xl = w, *xr = xl + x->len, *xu = xr + x->len;
    float *yl = xu + x->len, *yr = yl + y->len, *yu = yr + y->len;
    orc_bpla_weights(x, xl, xr, xu);
    orc_bpla_weights(y, yl, yr, yu);
    S.xl = xl; S.xr = xr; S.xu = xu; S.yl = yl; S.yr = yr; S.yu = yu;
  }
  double r = sw ? bpla_max(&S, gap, ext) : bpla_exp(&S, beta, gap, ext);
  free(w);
  return r;
}

/* ---- BPLA gradients (the bpla_optimizer's per-pair step) ----------------
 * BPLAKernel::compute_gradients (bpla_kernel/bpla_kernel.cpp:385-401):
 * BPLA_Forward (:178-243) and BPLA_Backward (:245-305) over the states
 * M, IX, IY, LX, LY, RX, RY, then BPLA_ForwardBackword (:325-383), which sums
 * d(value)/d(alpha, beta, gap, ext) over the cells.  Scores are
 * alpha*(pr*pr' + pl*pl') + pu*pu'*LAScore with the float products as written.
 * Returns the forward value 1 + M + RX + RY at (|x|, |y|). */
enum { G_M = 0, G_IX, G_IY, G_LX, G_LY, G_RX, G_RY, G_N };

double orc_bpla_gradients(const orc_mdata *x, const orc_mdata *y, double alpha, double beta,
                          double gap, double ext, const double *table16, double *d4) {
  if (!x->bpp || !y->bpp) return NAN; /* the reference indexes empty vectors */
  la_score S;
  memset(&S, 0, sizeof(S));
  S.x = x;
  S.y = y;
  S.table = table16;
  const int n = x->len, m = y->len, W = m + 1;
  float *w = (float *)malloc(sizeof(float) * 3 * (size_t)(n + m + 1));
  float *xl = w, *xr = xl + n, *xu = xr + n, *yl = xu + n, *yr = yl + m, *yu = yr + m;
  orc_bpla_weights(x, xl, xr, xu);
  orc_bpla_weights(y, yl, yr, yu);
  const size_t cells = (size_t)(n + 1) * (m + 1);
  double *F = (double *)calloc(G_N * cells, sizeof(double));
  double *B = (double *)calloc(G_N * cells, sizeof(double));
#define T3(T, s, i, j) T[(size_t)(s) * cells + (size_t)(i) * W + (j)]
  const double beta_gap = exp(beta * gap), beta_ext = exp(beta * ext);
  /* BPLA_Forward */
  T3(F, G_M, 0, 0) = 1;
  T3(F, G_LX, 0, 0) = 1;
  T3(F, G_LY, 0, 0) = 1;
  for (int i = 1; i <= n; ++i) T3(F, G_LX, i, 0) += T3(F, G_LX, i - 1, 0);
  for (int j = 1; j <= m; ++j) T3(F, G_LY, 0, j) += T3(F, G_LY, 0, j - 1);
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      const double s = alpha * (double)(xr[i - 1] * yr[j - 1] + xl[i - 1] * yl[j - 1]) +
                       (double)(xu[i - 1] * yu[j - 1]) * la_score_fn(&S, i - 1, j - 1);
      const double bs = exp(beta * s);
      T3(F, G_M, i, j) += bs * T3(F, G_M, i - 1, j - 1);
      T3(F, G_M, i, j) += bs * T3(F, G_IX, i - 1, j - 1);
      T3(F, G_M, i, j) += bs * T3(F, G_IY, i - 1, j - 1);
      T3(F, G_M, i, j) += bs * T3(F, G_LX, i - 1, j - 1);
      T3(F, G_M, i, j) += bs * T3(F, G_LY, i - 1, j - 1);
      T3(F, G_IX, i, j) += beta_gap * T3(F, G_M, i - 1, j);
      T3(F, G_IX, i, j) += beta_ext * T3(F, G_IX, i - 1, j);
      T3(F, G_IY, i, j) += beta_gap * T3(F, G_M, i, j - 1);
      T3(F, G_IY, i, j) += beta_gap * T3(F, G_IX, i, j - 1);
      T3(F, G_IY, i, j) += beta_ext * T3(F, G_IY, i, j - 1);
      T3(F, G_LX, i, j) += T3(F, G_LX, i - 1, 0);
      T3(F, G_LY, i, j) += T3(F, G_LX, i, j - 1);
      T3(F, G_LY, i, j) += T3(F, G_LY, i, j - 1);
      T3(F, G_RX, i, j) += T3(F, G_M, i - 1, j);
      T3(F, G_RX, i, j) += T3(F, G_RX, i - 1, j);
      T3(F, G_RY, i, j) += T3(F, G_M, i, j - 1);
      T3(F, G_RY, i, j) += T3(F, G_RX, i, j - 1);
      T3(F, G_RY, i, j) += T3(F, G_RY, i, j - 1);
    }
  /* BPLA_Backward */
  T3(B, G_M, n, m) = 1;
  T3(B, G_RX, n, m) = 1;
  T3(B, G_RY, n, m) = 1;
  for (int i = n; i != 0; --i)
    for (int j = m; j != 0; --j) {
      const double s = alpha * (double)(xr[i - 1] * yr[j - 1] + xl[i - 1] * yl[j - 1]) +
                       (double)(xu[i - 1] * yu[j - 1]) * la_score_fn(&S, i - 1, j - 1);
      const double bs = exp(beta * s);
      T3(B, G_M, i - 1, j - 1) += bs * T3(B, G_M, i, j);
      T3(B, G_IX, i - 1, j - 1) += bs * T3(B, G_M, i, j);
      T3(B, G_IY, i - 1, j - 1) += bs * T3(B, G_M, i, j);
      T3(B, G_LX, i - 1, j - 1) += bs * T3(B, G_M, i, j);
      T3(B, G_LY, i - 1, j - 1) += bs * T3(B, G_M, i, j);
      T3(B, G_M, i - 1, j) += beta_gap * T3(B, G_IX, i, j);
      T3(B, G_IX, i - 1, j) += beta_ext * T3(B, G_IX, i, j);
      T3(B, G_M, i, j - 1) += beta_gap * T3(B, G_IY, i, j);
      T3(B, G_IX, i, j - 1) += beta_gap * T3(B, G_IY, i, j);
      T3(B, G_IY, i, j - 1) += beta_ext * T3(B, G_IY, i, j);
      T3(B, G_LX, i - 1, 0) += T3(B, G_LX, i, j);
      T3(B, G_LX, i, j - 1) += T3(B, G_LY, i, j);
      T3(B, G_LY, i, j - 1) += T3(B, G_LY, i, j);
      T3(B, G_M, i - 1, j) += T3(B, G_RX, i, j);
      T3(B, G_RX, i - 1, j) += T3(B, G_RX, i, j);
      T3(B, G_M, i, j - 1) += T3(B, G_RY, i, j);
      T3(B, G_RX, i, j - 1) += T3(B, G_RY, i, j);
      T3(B, G_RY, i, j - 1) += T3(B, G_RY, i, j);
    }
  for (int i = n; i != 0; --i) T3(B, G_LX, i - 1, 0) += T3(B, G_LX, i, 0);
  for (int j = m; j != 0; --j) T3(B, G_LY, 0, j - 1) += T3(B, G_LY, 0, j);
  /* BPLA_ForwardBackword: update_alpha_beta (:307-314), update_beta_gap_ext (:316-323) */
  double da = 0.0, db = 0.0, dg = 0.0, de = 0.0;
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      const double wp = (double)(xr[i - 1] * yr[j - 1] + xl[i - 1] * yl[j - 1]);
      const double wu = (double)(xu[i - 1] * yu[j - 1]) * la_score_fn(&S, i - 1, j - 1);
      const double bs = exp(beta * (alpha * wp + wu));
      const double bm = T3(B, G_M, i, j);
      const int src[5] = {G_M, G_IX, G_IY, G_LX, G_LY};
      for (int t = 0; t < 5; ++t) {
        const double v = T3(F, src[t], i - 1, j - 1) * bs * bm;
        da += beta * wp * v;
        db += (alpha * wp + wu) * v;
      }
      double v = T3(F, G_M, i - 1, j) * beta_gap * T3(B, G_IX, i, j);
      db += gap * v, dg += beta * v;
      v = T3(F, G_IX, i - 1, j) * beta_ext * T3(B, G_IX, i, j);
      db += ext * v, de += beta * v;
      v = T3(F, G_M, i, j - 1) * beta_gap * T3(B, G_IY, i, j);
      db += gap * v, dg += beta * v;
      v = T3(F, G_IX, i, j - 1) * beta_gap * T3(B, G_IY, i, j);
      db += gap * v, dg += beta * v;
      v = T3(F, G_IY, i, j - 1) * beta_ext * T3(B, G_IY, i, j);
      db += ext * v, de += beta * v;
    }
  const double r = 1 + T3(F, G_M, n, m) + T3(F, G_RX, n, m) + T3(F, G_RY, n, m);
  d4[0] = da, d4[1] = db, d4[2] = dg, d4[3] = de;
  /* the backward pass's own total (1 + M + LX + LY at (0,0)) is the same
   * partition function: d4[4] reports it as a consistency check */
  d4[4] = 1 + T3(B, G_M, 0, 0) + T3(B, G_LX, 0, 0) + T3(B, G_LY, 0, 0);
#undef T3
  free(F);
  free(B);
  free(w);
  return r;
}

/* ------------------------------------------------------------------ */
/* 4-D stem kernel: StemKernel<double,BPMat>::full_dp
 * (stem_kernel/stem_kernel.cpp:282-351) with dp_init / dp_update (:85-111).
 * BPMat::prob (:354-421): model 0 = BPMatrix (Vienna pr via PFWrapper; here
 * the caller's matrix, prob(i,i) = 0), 1 = NormalBasePair, 2 = WobbleBasePair.
 * Sequences are compared as given (the loader lowercases, example.cpp:33). */
typedef struct {
  const char *s;
  const double *bpp; /* strict upper, packed (model 0) */
  int n, model;
  unsigned loop;
} bp4;

static float bp4_prob(const bp4 *B, int i, int j) {
  if (B->model == 0) return i < j ? (float)B->bpp[tri_index(B->n, i, j)] : 0.0f;
  const char a = B->s[i], b = B->s[j];
  int ok = (a == 'a' && b == 'u') || (a == 'u' && b == 'a') || (a == 'g' && b == 'c') ||
           (a == 'c' && b == 'g');
  if (B->model == 2) ok = ok || (a == 'g' && b == 'u') || (a == 'u' && b == 'g');
  return ((unsigned)i + 1 + B->loop <= (unsigned)j && ok) ? 1.0f : 0.0f;
}

enum { S_K0 = 0, S_K1, S_K2, S_K3, S_G0, S_G1, S_G2, S_G3 };

/* srcsum (may be NULL): the sum of every stacking source the K3 updates add
 * (:327-331), in the reference's loop order -- 1 + srcsum is the K-sum
 * formulation of the engine's full_dp kernel, checked against
 * K0(0,n,0,m) of the chain itself (tests/test_stem4d.py) */
static double stem4d_full(const char *x, const double *bpx, const char *y, const double *bpy,
                          double gap, double stack, double subst, float bp_bound, int model,
                          unsigned loop, double *srcsum) {
  const int n = (int)strlen(x), m = (int)strlen(y);
  double ssum = 0.0;
  const double g = gap;
  bp4 BX = {x, bpx, n, model, loop}, BY = {y, bpy, m, model, loop};
  /* planes (i,j) of columns j-1 and j; cell (k,l), k<=l, triangular */
  const size_t cells = (size_t)(m + 1) * (m + 2) / 2;
  const size_t plane = cells * 8;
#define CELL(k, l) ((size_t)(l) * ((l) + 1) / 2 + (size_t)(k))
  double *col[2];
  col[0] = (double *)calloc((size_t)(n + 1) * plane, sizeof(double));
  col[1] = (double *)calloc((size_t)(n + 1) * plane, sizeof(double));
  double result = 0.0;
  for (int j = 0; j <= n; ++j) {
    double *cur = col[j & 1], *prv = col[(j + 1) & 1];
#define DP(C, s, i, k, l) ((C)[(size_t)(i) * plane + (size_t)(s) * cells + CELL(k, l)])
    /* plane (j,j): K0 = 1, others 0, G0(k,l) = G0(k+1,l)*g */
    memset(&cur[(size_t)j * plane], 0, plane * sizeof(double));
    for (size_t c = 0; c < cells; ++c) cur[(size_t)j * plane + S_K0 * cells + c] = 1.0;
    for (int l = 0; l <= m; ++l) {
      DP(cur, S_G0, j, l, l) = 1.0;
      for (int k = l - 1; k >= 0; --k) DP(cur, S_G0, j, k, l) = DP(cur, S_G0, j, k + 1, l) * g;
    }
    for (int i = j - 1; i >= 0; --i) {
      const float bp_ij = bp4_prob(&BX, i, j - 1);
      memset(&cur[(size_t)i * plane], 0, plane * sizeof(double));
      for (int l = 0; l <= m; ++l) {
        DP(cur, S_K0, i, l, l) = 1.0;
        DP(cur, S_G0, i, l, l) = DP(cur, S_G0, i + 1, l, l) * g;
        for (int k = l - 1; k >= 0; --k) {
          /* dp_init (:85-96) */
          DP(cur, S_K0, i, k, l) = DP(prv, S_K0, i, k, l);
          DP(cur, S_G0, i, k, l) = DP(prv, S_G0, i, k, l) * g;
          DP(cur, S_K1, i, k, l) = DP(cur, S_K1, i + 1, k, l);
          DP(cur, S_G1, i, k, l) = DP(cur, S_G1, i + 1, k, l) * g;
          DP(cur, S_K2, i, k, l) = DP(cur, S_K2, i, k, l - 1);
          DP(cur, S_G2, i, k, l) = DP(cur, S_G2, i, k, l - 1) * g;
          DP(cur, S_K3, i, k, l) = DP(cur, S_K3, i, k + 1, l);
          DP(cur, S_G3, i, k, l) = DP(cur, S_G3, i, k + 1, l) * g;
          if (bp_ij > bp_bound) { /* :327-340 */
            const float bp_kl = bp4_prob(&BY, k, l - 1);
            if (bp_kl > bp_bound) {
              const double g0 = DP(prv, S_G0, i + 1, k + 1, l - 1);
              if (x[i] == y[k] && x[j - 1] == y[l - 1]) {
                DP(cur, S_K3, i, k, l) += g0 * stack * bp_ij * bp_kl;
                DP(cur, S_G3, i, k, l) += g0;
                ssum += g0 * stack * bp_ij * bp_kl;
              } else {
                DP(cur, S_K3, i, k, l) += g0 * stack * subst * bp_ij * bp_kl;
                ssum += g0 * stack * subst * bp_ij * bp_kl;
              }
            }
          }
          /* dp_update (:98-111) */
          DP(cur, S_K2, i, k, l) += DP(cur, S_K3, i, k, l);
          DP(cur, S_G2, i, k, l) += DP(cur, S_G3, i, k, l);
          DP(cur, S_K1, i, k, l) += DP(cur, S_K2, i, k, l);
          DP(cur, S_G1, i, k, l) += DP(cur, S_G2, i, k, l);
          DP(cur, S_K0, i, k, l) += DP(cur, S_K1, i, k, l);
          DP(cur, S_G0, i, k, l) += DP(cur, S_G1, i, k, l);
        }
      }
    }
    if (j == n) result = DP(cur, S_K0, 0, 0, m);
#undef DP
  }
#undef CELL
  free(col[0]);
  free(col[1]);
  if (srcsum) *srcsum = ssum;
  return result;
}

double orc_stem4d(const char *x, const double *bpx, const char *y, const double *bpy,
                  double gap, double stack, double subst, float bp_bound, int model,
                  unsigned loop) {
  return stem4d_full(x, bpx, y, bpy, gap, stack, subst, bp_bound, model, loop, NULL);
}

/* 1 + the sum of the stacking sources (the K-sum formulation) */
double orc_stem4d_ksum(const char *x, const double *bpx, const char *y, const double *bpy,
                       double gap, double stack, double subst, float bp_bound, int model,
                       unsigned loop) {
  double ssum = 0.0;
  stem4d_full(x, bpx, y, bpy, gap, stack, subst, bp_bound, model, loop, &ssum);
  return 1.0 + ssum;
}

/* Band constraints of StemKernel::alignment_constraints without alignment
 * posteriors (ali_bound == 0, band > 0; stem_kernel/stem_kernel.cpp:66-72). */
void orc_stem4d_band(int n, int m, unsigned band, unsigned *c_low, unsigned *c_high) {
  for (int i = 0; i <= n; ++i) {
    const unsigned j = (unsigned)((double)i / n * m + 0.5);
    c_low[i] = j < band ? 0u : j - band;
    c_high[i] = j + band > (unsigned)m ? (unsigned)m : j + band;
  }
}

/* ---- PairHMM alignment constraints (the 4-D kernel's -a option) ----------
 * PairHMM<Ribosum> of stem_kernel/phmm.cpp over LogValue<double>
 * (stem_kernel/log_value.h).  A LogValue holds log(v); products add logs
 * (:128-189); += is the branchy log-sum of :212-224 with log1exp0 the
 * probcons polynomial, FAST_LOG1EXP0 being defined at log_value.h:28
 * (:312-347).  zerop(LogValue) is `std::isinf(x.log())<0` (:374-378): with a
 * C++11 <cmath> std::isinf returns bool, so the test is always false and
 * every += onto log(0) = -inf yields NaN (-inf + log1exp0(+inf) = -inf+inf).
 * zerop_fixed = 0 reproduces that (the reference as g++ >= 6 builds it);
 * zerop_fixed = 1 gives the intended -inf test. */
enum { PH_M = 0, PH_IX = 1, PH_IY = 2 };

/* ribosum_trans / ribosum_emit, phmm.cpp:262-276, stored as logs (ExpOf) */
static const double kPhTrans[3][3] = {{0.0, -5.0, -5.0}, {-10.0, -5.0, -15.0}, {-10.0, -5.0, -15.0}};
static const double kPhEmit[4][4] = {{2.22, -1.86, -1.46, -1.39},
                                     {-1.86, 1.16, -2.48, -1.05},
                                     {-1.46, -2.48, 1.03, -1.74},
                                     {-1.39, -1.05, -1.74, 1.65}};

/* log_value.h:312-347 with FAST_LOG1EXP0 */
static double lv_log1exp0(double x) {
  if (x > 10.0f) return x;
  if (x >= 0.00f) {
    if (x <= 1.00f)
      return ((-0.009350833524763f * x + 0.130659527668286f) * x + 0.498799810682272f) * x +
             0.693203116424741f;
    if (x <= 2.50f)
      return ((-0.014532321752540f * x + 0.139942324101744f) * x + 0.495635523139337f) * x +
             0.692140569840976f;
    if (x <= 4.50f)
      return ((-0.004605031767994f * x + 0.063427417320019f) * x + 0.695956496475118f) * x +
             0.514272634594009f;
    if (x <= 7.50f)
      return ((-0.000458661602210f * x + 0.009695946122598f) * x + 0.930734667215156f) * x +
             0.168037164329057f;
    return (((0.00000051726300753785 * x - 0.00002720671238876090) * x + 0.00053403733818413500) * x +
            0.99536021775747900000) * x + 0.01507065715532010000;
  }
  return log(exp(x) + 1.0);
}

static int lv_zerop(double v, int fixed) { return fixed && isinf(v) && v < 0; }

/* LogValue::operator+= (log_value.h:212-224) */
static void lv_addto(double *a, double b, int fixed) {
  if (lv_zerop(b, fixed)) return;
  if (lv_zerop(*a, fixed)) {
    *a = b;
    return;
  }
  if (*a < b)
    *a += lv_log1exp0(b - *a);
  else
    *a = b + lv_log1exp0(*a - b);
}

/* char2rna of phmm.cpp:247-258 (asserts on anything but ACGU) */
static int ph_base(char c) {
  switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 'u': case 'U': return 3;
  }
  return -1;
}

#define PH(T, s, i, j) ((T)[((size_t)(s) * (n + 1) + (size_t)(i)) * (m + 1) + (size_t)(j)])

/* PairHMM::forward_backward (phmm.cpp:10-50 forward, :52-93 backward,
 * :95-115 posterior fw*bk/w); fb: 3*(n+1)*(m+1) doubles.  Returns -1 on a
 * non-ACGU residue (the reference asserts). */
int orc_phmm_posterior(const char *x, const char *y, int fixed, double *fb) {
  const int n = (int)strlen(x), m = (int)strlen(y);
  for (int i = 0; i < n; ++i)
    if (ph_base(x[i]) < 0) return -1;
  for (int j = 0; j < m; ++j)
    if (ph_base(y[j]) < 0) return -1;
  const size_t cells = (size_t)3 * (n + 1) * (m + 1);
  double *fw = (double *)malloc(cells * sizeof(double));
  double *bk = (double *)malloc(cells * sizeof(double));
  const double z = log(0.0); /* LogValue(0.0) */
  for (size_t c = 0; c < cells; ++c) fw[c] = bk[c] = z;
  /* forward */
  PH(fw, PH_M, 0, 0) = log(1.0);
  for (int i = 1; i <= n; ++i) {
    PH(fw, PH_M, i, 0) = PH(fw, PH_IY, i, 0) = z;
    for (int s = 0; s < 3; ++s) lv_addto(&PH(fw, PH_IX, i, 0), PH(fw, s, i - 1, 0) + kPhTrans[s][PH_IX], fixed);
  }
  for (int j = 1; j <= m; ++j) {
    PH(fw, PH_M, 0, j) = PH(fw, PH_IX, 0, j) = z;
    for (int s = 0; s < 3; ++s) lv_addto(&PH(fw, PH_IY, 0, j), PH(fw, s, 0, j - 1) + kPhTrans[s][PH_IY], fixed);
  }
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      const double e = kPhEmit[ph_base(x[i - 1])][ph_base(y[j - 1])];
      for (int s = 0; s < 3; ++s) {
        lv_addto(&PH(fw, PH_M, i, j), PH(fw, s, i - 1, j - 1) + (kPhTrans[s][PH_M] + e), fixed);
        lv_addto(&PH(fw, PH_IX, i, j), PH(fw, s, i - 1, j) + kPhTrans[s][PH_IX], fixed);
        lv_addto(&PH(fw, PH_IY, i, j), PH(fw, s, i, j - 1) + kPhTrans[s][PH_IY], fixed);
      }
    }
  /* backward */
  PH(bk, PH_M, n, m) = log(1.0);
  for (int i = n; i != 0; --i)
    for (int j = m; j != 0; --j) {
      const double e = kPhEmit[ph_base(x[i - 1])][ph_base(y[j - 1])];
      for (int s = 0; s < 3; ++s) {
        lv_addto(&PH(bk, s, i - 1, j - 1), PH(bk, PH_M, i, j) + (kPhTrans[s][PH_M] + e), fixed);
        lv_addto(&PH(bk, s, i - 1, j), PH(bk, PH_IX, i, j) + kPhTrans[s][PH_IX], fixed);
        lv_addto(&PH(bk, s, i, j - 1), PH(bk, PH_IY, i, j) + kPhTrans[s][PH_IY], fixed);
      }
    }
  for (int j = m; j != 0; --j) {
    PH(bk, PH_M, 0, j) = PH(bk, PH_IX, 0, j) = z;
    for (int s = 0; s < 3; ++s) lv_addto(&PH(bk, s, 0, j - 1), PH(bk, PH_IY, 0, j) + kPhTrans[s][PH_IY], fixed);
  }
  for (int i = n; i != 0; --i) {
    PH(bk, PH_M, i, 0) = PH(bk, PH_IY, i, 0) = z;
    for (int s = 0; s < 3; ++s) lv_addto(&PH(bk, s, i - 1, 0), PH(bk, PH_IX, i, 0) + kPhTrans[s][PH_IX], fixed);
  }
  /* posterior: LogValue fw*bk/w converted to double (exp) */
  const double w = PH(fw, PH_M, n, m);
  for (size_t c = 0; c < cells; ++c) fb[c] = exp((fw[c] + bk[c]) - w);
  free(fw);
  free(bk);
  return 0;
}

/* StemKernel::alignment_constraints (stem_kernel/stem_kernel.cpp:14-81):
 * posteriors, MAP path by PairHMM::forward(fb,tr) + traceback
 * (phmm.cpp:117-236), anchors = M positions of the path with posterior >=
 * ali_bound, then the band widening.  c_low/c_high: n+1 entries. */
int orc_alignment_constraints(const char *x, const char *y, float ali_bound, unsigned band,
                              int fixed, unsigned *c_low, unsigned *c_high) {
  const int n = (int)strlen(x), m = (int)strlen(y);
  for (int i = 0; i <= n; ++i) {
    c_low[i] = 0;
    c_high[i] = (unsigned)m;
  }
  if (ali_bound > 0.0) {
    const size_t cells = (size_t)3 * (n + 1) * (m + 1);
    double *fb = (double *)malloc(cells * sizeof(double));
    if (orc_phmm_posterior(x, y, fixed, fb)) {
      free(fb);
      return -1;
    }
    double *mf = (double *)calloc(cells, sizeof(double));
    unsigned *tr = (unsigned *)malloc(cells * sizeof(unsigned));
    for (size_t c = 0; c < cells; ++c) tr[c] = (unsigned)-1;
    for (int s = 0; s < 3; ++s) PH(mf, s, 0, 0) = PH(fb, s, 0, 0);
#define PH_UPD(S, I, J, V, FROM)                                             \
  do {                                                                       \
    const double v_ = (V);                                                   \
    if (PH(tr, S, I, J) == (unsigned)-1 || PH(mf, S, I, J) < v_) {           \
      PH(mf, S, I, J) = v_;                                                  \
      PH(tr, S, I, J) = (FROM);                                              \
    }                                                                        \
  } while (0)
    for (int i = 1; i <= n; ++i) {
      PH(mf, PH_M, i, 0) = PH(mf, PH_IY, i, 0) = 0.0;
      for (int s = 0; s < 3; ++s) PH_UPD(PH_IX, i, 0, PH(mf, s, i - 1, 0) + PH(fb, PH_IX, i, 0), s);
    }
    for (int j = 1; j <= m; ++j) {
      PH(mf, PH_M, 0, j) = PH(mf, PH_IX, 0, j) = 0.0;
      for (int s = 0; s < 3; ++s) PH_UPD(PH_IY, 0, j, PH(mf, s, 0, j - 1) + PH(fb, PH_IY, 0, j), s);
    }
    for (int i = 1; i <= n; ++i)
      for (int j = 1; j <= m; ++j)
        for (int s = 0; s < 3; ++s) {
          PH_UPD(PH_M, i, j, PH(mf, s, i - 1, j - 1) + PH(fb, PH_M, i, j), s);
          PH_UPD(PH_IX, i, j, PH(mf, s, i - 1, j) + PH(fb, PH_IX, i, j), s);
          PH_UPD(PH_IY, i, j, PH(mf, s, i, j - 1) + PH(fb, PH_IY, i, j), s);
        }
#undef PH_UPD
    /* traceback (phmm.cpp:187-216): path from (M,n,m) back to row/column 0 */
    int *ps = (int *)malloc(sizeof(int) * 3 * (n + m + 2));
    int len = 0, s = PH_M, px = n, py = m;
    ps[0] = s, ps[1] = px, ps[2] = py, len = 1;
    while (px != 0 && py != 0) {
      const unsigned t = PH(tr, s, px, py);
      if (s == PH_M) --px, --py;
      else if (s == PH_IX) --px;
      else --py;
      s = (int)t;
      ps[3 * len] = s, ps[3 * len + 1] = px, ps[3 * len + 2] = py, ++len;
    }
    /* anchors, in path order (:40-57) */
    unsigned low_x = 0, low_y = 0;
    for (int k = len - 1; k >= 0; --k) {
      const int S = ps[3 * k], X = ps[3 * k + 1], Y = ps[3 * k + 2];
      if (S == PH_M && PH(fb, PH_M, X, Y) >= ali_bound) {
        for (unsigned i = low_x; i != (unsigned)X; ++i) {
          c_low[i] = low_y;
          c_high[i] = (unsigned)Y;
        }
        c_low[X] = (unsigned)Y;
        c_high[X] = (unsigned)Y;
        low_x = (unsigned)X + 1;
        low_y = (unsigned)Y;
      }
    }
    for (unsigned i = low_x; i != (unsigned)n + 1; ++i) {
      c_low[i] = low_y;
      c_high[i] = (unsigned)m;
    }
    if (band > 0)
      for (int i = 0; i <= n; ++i)
        if (c_high[i] - c_low[i] < band * 2) {
          const unsigned j = (c_high[i] + c_low[i]) / 2;
          c_low[i] = j < band ? 0 : j - band;
          c_high[i] = j + band > (unsigned)m ? (unsigned)m : j + band;
        }
    free(ps);
    free(tr);
    free(mf);
    free(fb);
  } else if (band > 0) {
    orc_stem4d_band(n, m, band, c_low, c_high);
  }
  return 0;
}
#undef PH

/* StemKernel<double,BPMat>::partial_dp (stem_kernel/stem_kernel.cpp:113-280):
 * cells outside the constraints stay at the planes' zero fill; K0 past
 * c_high[j-1] and K1 below c_low[i+1] use the reference's boundary
 * approximations.  Band-only (-b) constraints. */
double orc_stem4d_banded(const char *x, const double *bpx, const char *y, const double *bpy,
                         double gap, double stack, double subst, float bp_bound, int model,
                         unsigned loop, unsigned band) {
  return orc_stem4d_partial(x, bpx, y, bpy, gap, stack, subst, bp_bound, model, loop, band, 0.0f, 0);
}

/* partial_dp with the constraints of alignment_constraints(ali_bound, band);
 * NaN when a constrained pair holds a non-ACGU residue (the reference asserts). */
double orc_stem4d_partial(const char *x, const double *bpx, const char *y, const double *bpy,
                          double gap, double stack, double subst, float bp_bound, int model,
                          unsigned loop, unsigned band, float ali_bound, int zerop_fixed) {
  const int n = (int)strlen(x), m = (int)strlen(y);
  const double g = gap;
  bp4 BX = {x, bpx, n, model, loop}, BY = {y, bpy, m, model, loop};
  unsigned *cl = (unsigned *)malloc(sizeof(unsigned) * (n + 1));
  unsigned *chh = (unsigned *)malloc(sizeof(unsigned) * (n + 1));
  /* alignment_constraints runs first (:126) */
  const int bad = orc_alignment_constraints(x, y, ali_bound, band, zerop_fixed, cl, chh);
  if (bad || n == 0) {
    free(cl);
    free(chh);
    return bad ? NAN : 1.0; /* n == 0: K0(0,0,0,m) of the initialised plane (0,0) */
  }
  double *gpw = (double *)malloc(sizeof(double) * (m + 1));
  gpw[0] = 1.0;
  for (int i = 1; i <= m; ++i) gpw[i] = gpw[i - 1] * g;
  const size_t cells = (size_t)(m + 1) * (m + 2) / 2;
  const size_t plane = cells * 8;
#define CELL(k, l) ((size_t)(l) * ((l) + 1) / 2 + (size_t)(k))
  double *col[2];
  col[0] = (double *)calloc((size_t)(n + 1) * plane, sizeof(double));
  col[1] = (double *)calloc((size_t)(n + 1) * plane, sizeof(double));
  double result = 0.0;
  for (int j = 0; j <= n; ++j) {
    double *cur = col[j & 1], *prv = col[(j + 1) & 1];
#define DP(C, s, i, k, l) ((C)[(size_t)(i) * plane + (size_t)(s) * cells + CELL(k, l)])
    memset(&cur[(size_t)j * plane], 0, plane * sizeof(double));
    for (size_t c = 0; c < cells; ++c) cur[(size_t)j * plane + S_K0 * cells + c] = 1.0;
    for (int l = 0; l <= m; ++l) {
      DP(cur, S_G0, j, l, l) = 1.0;
      for (int k = l - 1; k >= 0; --k) DP(cur, S_G0, j, k, l) = DP(cur, S_G0, j, k + 1, l) * g;
    }
    for (int i = j - 1; i >= 0; --i) {
      const float bp_ij = bp4_prob(&BX, i, j - 1);
      memset(&cur[(size_t)i * plane], 0, plane * sizeof(double));
      for (int l = (int)cl[j]; l <= (int)chh[j]; ++l) {
        DP(cur, S_K0, i, l, l) = 1.0;
        DP(cur, S_G0, i, l, l) = DP(cur, S_G0, i + 1, l, l) * g;
        if (l == 0) continue;
        const int kt = (l - 1) < (int)chh[i] ? (l - 1) : (int)chh[i];
        for (int k = kt; k >= (int)cl[i]; --k) {
          if (l <= (int)chh[j - 1]) {
            DP(cur, S_K0, i, k, l) = DP(prv, S_K0, i, k, l);
            DP(cur, S_G0, i, k, l) = DP(prv, S_G0, i, k, l) * g;
          } else { /* approximation (:183-186) */
            DP(cur, S_K0, i, k, l) = DP(prv, S_K0, i, k, chh[j - 1]);
            DP(cur, S_G0, i, k, l) = DP(prv, S_G0, i, k, chh[j - 1]) * g * g;
          }
          if (k >= (int)cl[i + 1]) {
            DP(cur, S_K1, i, k, l) = DP(cur, S_K1, i + 1, k, l);
            DP(cur, S_G1, i, k, l) = DP(cur, S_G1, i + 1, k, l) * g;
          } else { /* approximation (:193-196) */
            DP(cur, S_K1, i, k, l) = DP(cur, S_K1, i + 1, cl[i + 1], l);
            DP(cur, S_G1, i, k, l) = DP(cur, S_G1, i + 1, cl[i + 1], l) * g * g;
          }
          if (l - 1 >= (int)cl[j] || k == l - 1) {
            DP(cur, S_K2, i, k, l) = DP(cur, S_K2, i, k, l - 1);
            DP(cur, S_G2, i, k, l) = DP(cur, S_G2, i, k, l - 1) * g;
          } else { /* :221-227 */
            DP(cur, S_K2, i, k, l) = 0.0;
            DP(cur, S_G2, i, k, l) = 0.0;
            for (int ll = k; ll != l; ++ll) {
              DP(cur, S_K2, i, k, l) += DP(cur, S_K3, i, ll, ll);
              DP(cur, S_G2, i, k, l) += DP(cur, S_G3, i, ll, ll) * gpw[l - k];
            }
          }
          if (k + 1 <= (int)chh[i]) {
            DP(cur, S_K3, i, k, l) = DP(cur, S_K3, i, k + 1, l);
            DP(cur, S_G3, i, k, l) = DP(cur, S_G3, i, k + 1, l) * g;
          } else { /* :233-235 */
            DP(cur, S_K3, i, k, l) = DP(cur, S_K3, i, l, l);
            DP(cur, S_G3, i, k, l) = DP(cur, S_G3, i, l, l) * gpw[l - k];
          }
          if (bp_ij > bp_bound) {
            const float bp_kl = bp4_prob(&BY, k, l - 1);
            if (bp_kl > bp_bound) {
              const double g0 = DP(prv, S_G0, i + 1, k + 1, l - 1);
              if (x[i] == y[k] && x[j - 1] == y[l - 1]) {
                DP(cur, S_K3, i, k, l) += g0 * stack * bp_ij * bp_kl;
                DP(cur, S_G3, i, k, l) += g0;
              } else {
                DP(cur, S_K3, i, k, l) += g0 * stack * subst * bp_ij * bp_kl;
              }
            }
          }
          DP(cur, S_K2, i, k, l) += DP(cur, S_K3, i, k, l);
          DP(cur, S_G2, i, k, l) += DP(cur, S_G3, i, k, l);
          DP(cur, S_K1, i, k, l) += DP(cur, S_K2, i, k, l);
          DP(cur, S_G1, i, k, l) += DP(cur, S_G2, i, k, l);
          DP(cur, S_K0, i, k, l) += DP(cur, S_K1, i, k, l);
          DP(cur, S_G0, i, k, l) += DP(cur, S_G1, i, k, l);
        }
      }
    }
    if (j == n) result = DP(cur, S_K0, 0, 0, m);
#undef DP
  }
#undef CELL
  free(col[0]);
  free(col[1]);
  free(cl);
  free(chh);
  free(gpw);
  return result;
}
