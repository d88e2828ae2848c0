// Loop energies of the McCaskill fold (fold.hip), dcal/mol at
// 37 C: the Turner-1999 core the legacy ViennaRNA library (>= 1.6, the
// reference's pf_fold, common/bpmatrix.cpp:151-177) compiles in -- stacks,
// hairpin / bulge / interior initiation (lxc extrapolation past 30), Ninio
// asymmetry, terminal AU/GU penalty, linear multiloop -- without its
// terminal-mismatch, dangle, special-hairpin and 1x1/1x2/2x2 tables (not in
// this image; parity against ViennaRNA is unpinned).
#pragma once

namespace sk {
namespace foldp {
constexpr double kT = (37.0 + 273.15) * 1.98717 / 10.0;  // dcal/mol
constexpr double lxc = 107.856;
// pair types CG=1 GC=2 GU=3 UG=4 AU=5 UA=6; [type(i,j)][type(q,p)]
constexpr int stack37[7][7] = {{0, 0, 0, 0, 0, 0, 0},
                               {0, -240, -330, -210, -140, -210, -210},
                               {0, -330, -340, -250, -150, -220, -240},
                               {0, -210, -250, 130, -50, -140, -130},
                               {0, -140, -150, -50, 30, -60, -100},
                               {0, -210, -220, -140, -60, -110, -90},
                               {0, -210, -240, -130, -100, -90, -130}};
constexpr int hairpin37[31] = {0,   0,   0,   570, 560, 560, 540, 590, 560, 640, 650,
                               660, 670, 678, 686, 694, 701, 707, 713, 719, 725, 730,
                               735, 740, 744, 749, 753, 757, 761, 765, 769};
constexpr int bulge37[31] = {0,   380, 280, 320, 360, 400, 440, 459, 470, 480, 490,
                             500, 510, 519, 527, 534, 541, 548, 554, 560, 565, 571,
                             576, 580, 585, 589, 594, 598, 602, 605, 609};
constexpr int interior37[31] = {0,   0,   410, 510, 170, 180, 200, 220, 230, 240, 250,
                                260, 270, 278, 286, 294, 301, 307, 313, 319, 325, 330,
                                335, 340, 345, 349, 353, 357, 361, 365, 369};
constexpr int ml_closing = 340, ml_intern = 40, terminal_au = 50, ninio = 50, max_ninio = 300;
constexpr int max_loop = 30;
// per-nucleotide scale: every subsequence's weight carries sc^len, sc =
// exp(log_sc), keeping Z within double range for lengths up to ~1,400
constexpr double log_sc = -0.35;
}  // namespace foldp
}  // namespace sk
