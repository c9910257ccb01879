/** \file layout.hpp
 * \brief Device data layout for the MI355X face sweep.
 *
 * Cells are renumbered internally along a Hilbert curve and cut into PATCHES: contiguous ranges
 * of internal cells whose touching faces number at most SLOTS_MAX. A patch is processed by one
 * workgroup: each face touching the patch gets a SLOT (faces shared by two patches are stored,
 * and computed, once per patch), its flux goes to LDS, and every cell then sums its faces from
 * LDS in ascending reference face index — the single-thread order of the reference's
 * `omp atomic` scatter (flow_spatial.cpp:552-561) — so residuals are deterministic and
 * reproduce the reference bit for bit. Exported indices are never changed.
 */
#ifndef FVHIP_LAYOUT_HPP
#define FVHIP_LAYOUT_HPP

#include <vector>
#include <cstdint>
#include "../../include/fvhip.h"

namespace fvhip {

#ifndef FVHIP_SLOTS
#define FVHIP_SLOTS 256
#endif
#ifndef FVHIP_FUSED_ROWS
#define FVHIP_FUSED_ROWS (FVHIP_SLOTS*11/8)   // 352 x 112 B = 39 KB for 256-slot patches: 4 blocks = 16 waves per CU, the VGPR-bound occupancy
#endif
constexpr int SLOTS_MAX = FVHIP_SLOTS;   ///< faces per patch = threads per sweep workgroup
constexpr int CELLS_MAX = FVHIP_SLOTS;
constexpr int MAXF = 4;          ///< max faces per cell (linear tri/quad)

struct Layout
{
	int ncell = 0;               ///< owned cells
	int nghost = 0;              ///< ghost cells (internal ids ncell .. ncell+nghost-1)
	int nbface = 0, naface = 0, ninface = 0;
	std::vector<int> perm;       ///< perm[internal] = reference cell
	std::vector<int> iperm;      ///< iperm[reference] = internal
	// patches
	std::vector<int> patch_cell;   ///< [npatch+1] start of each patch's cells (internal ids)
	std::vector<int> patch_slot;   ///< [npatch+1] start of each patch's slots
	// slots (patch order; faces touching two patches appear twice)
	std::vector<int> slot_L, slot_R;       ///< internal cell ids; R >= ncell: physical boundary R-ncell
	std::vector<int> slot_face;            ///< reference face index
	std::vector<double> slot_n;            ///< [S][2]
	std::vector<double> slot_len;          ///< [S]
	std::vector<double> slot_gr;           ///< [S][2]
	// cells (internal order)
	std::vector<int> cell_slots;           ///< [ncell][4]: (slot << 1 | cell-is-right) of the cell's
	                                       ///<  faces in ascending reference face index, -1 padded;
	                                       ///<  the slot is the copy in the cell's own patch
	std::vector<int> cell_nbr_local;       ///< [ncell][4]: esuel neighbours (internal or boundary
	                                       ///<  code ncell+bf) in local-face order (WENO, limiters)
	std::vector<int> cell_face_local;      ///< [ncell][4]: slot of local face j (own patch)
	std::vector<int> cell_nbr_fo;          ///< [ncell][4]: neighbour across each face in ascending
	                                       ///<  reference face index (internal / ncell+bf), -1 pad
	std::vector<int> cell_nfael;
	std::vector<double> rc;                ///< [ncell+nghost][2]
	std::vector<double> area;              ///< [ncell]
	std::vector<double> wls_V;             ///< [ncell][4] WLS inverse, row-major (if built)
	std::vector<double> venk_eps2;         ///< [ncell] (K*clength)^3 (if built)
	// boundary faces (reference order)
	std::vector<int> bf_L;                 ///< internal id of the boundary cell
	std::vector<int> bf_bc;                ///< index into the BC table
	std::vector<double> bf_n;              ///< [nb][2]
	std::vector<double> bf_rcbp;           ///< [nb][2]
	std::vector<int> bf_tag;               ///< [nb] boundary marker (gbtags(face,0))
	std::vector<double> bf_gr;             ///< [nb][2] face centre (node average, aspatial.cpp:53-61)
	// interior faces (reference order, for the Jacobian): internal L, R
	std::vector<int> if_L, if_R;
	std::vector<int> if_slot;              ///< one slot carrying the face's geometry
	std::vector<double> if_n, if_len;      ///< [Fi][2], [Fi]
	std::vector<double> bf_len;            ///< [nb]
	std::vector<int> cell_rfaces;          ///< [ncell][4]: (reference face << 1 | cell-is-right),
	                                       ///<  same order as cell_slots
	int max_slots = 0;
	// halo (partitioned meshes): ghosts from nbr_rank[k] are internal cells
	// ncell+ghost_start[k] .. ncell+ghost_start[k+1]-1; send_cells[send_start[k]..] go to nbr_rank[k]
	std::vector<int> nbr_rank, ghost_start, send_start, send_cells;
	std::vector<int> border_cells;         ///< unique layer-1 send cells (their gradients are computed first)
	// two-layer halo (partition.hpp MeshTopo): layer-1 then layer-2 rows in each neighbour's block
	int halo_layers = 1;
	std::vector<int> ghost_l1_end, send_l1_end;   ///< [nnbr]
	std::vector<int> gg_cells;             ///< layer-1 ghosts whose gradients this rank computes
	std::vector<int> gg_nbr;               ///< [n1][4] internal neighbour, -2-j extra boundary face, -1
	std::vector<double> gg_V;              ///< [n1][4] their WLS inverses (as wls_V)
	std::vector<double> gg_gp;             ///< [n1][4][2] their face centres in gg_nbr order (limited
	                                       ///<  reconstructions: the ghosts' limiter values are local too)
	std::vector<double> gg_eps2;           ///< [n1] Venkatakrishnan (K*clength)^3 of each
	std::vector<int> xb_bc;                ///< extra boundary faces: BC index,
	std::vector<double> xb_n, xb_rcbp;     ///<  normal [2], ghost centre [2]
	std::vector<int> cell_global;          ///< [ncell+nghost] global cell of each internal cell
	std::vector<int> trace_conn;           ///< per-rank meshes: [nghost] the connectivity face (icface) of
	                                       ///<  each ghost entry = of each send entry (same order), for the
	                                       ///<  face-trace exchange (L2TraceVector)
	// fused residual (k_residual_wls): per patch, the ring-1 cells (far side of its cut faces) whose
	// primitive states and gradients it recomputes, and the ring-2 cells (the other neighbours of the
	// owned ring-1 cells) whose primitive states those gradients read; every cell a patch reads is
	// staged in LDS by one round of loads. Patch-local index = [patch cells | ring 1 | ring 2]
	std::vector<int> fz_ext_start;         ///< [npatch+1]
	std::vector<int> fz_ext;               ///< ring-1 then ring-2 cells of each patch (internal ids)
	std::vector<int> fz_n1;                ///< [npatch] ring-1 count
	std::vector<int> fz_g_start;           ///< [npatch+1] row offset of each patch's fz_gnbr rows
	std::vector<int> fz_gnbr;              ///< per patch [patch cells + ring 1][4]: neighbours in
	                                       ///<  ascending reference face order: patch-local index,
	                                       ///<  -2-bf (boundary face), -1 (none; also every entry of a
	                                       ///<  ghost ring-1 cell, whose gradient is received)
	std::vector<int> fz_slot_lr;           ///< [S][2] local L, R (R boundary: -2-bf)
	// the same, packed for the kernel (16-bit patch-local indices): per slot L | R << 16 with R = 0xFFFF
	// for a boundary face (its bf then comes from slot_R); per gradient row four neighbour codes
	// (0xFFFF none, 0x8000|j boundary face fz_gbf[fz_gbf_start[p] + j]); per owned cell its four faces
	// as (patch-local slot << 1 | isRight), 0xFFFF padded
	std::vector<uint32_t> fz_slot_lr16;    ///< [S]
	std::vector<uint16_t> fz_gnbr16;       ///< [rows][4], rows as fz_gnbr
	std::vector<int> fz_gbf_start;         ///< [npatch+1]
	std::vector<int> fz_gbf;               ///< boundary faces the gradient rows of each patch read
	std::vector<uint16_t> fz_cslot16;      ///< [ncell][4]
	int fz_ring2 = 0;                      ///< ring-2 cells staged over all patches
	int fz_max_cells = 0;
	int fz_row_cap = 0;                    ///< fusedRowCap of the configuration
	std::vector<int> fz_order;             ///< patches needing no halo data first (fz_ninner), then the rest
	int fz_ninner = 0;
	// pipelined staged residual (single domain, WLS): the gradient kernel runs in chunks of cells on
	// one stream while the sweep runs, on a second stream, the patches whose cells and halo cells
	// all lie in finished chunks; patches are grouped by the last chunk they read
	std::vector<int> pipe_cell_start;      ///< [K+1] gradient chunks (internal cell ranges)
	std::vector<int> pipe_patch;           ///< patches ordered by group, ascending index within one
	std::vector<int> pipe_group_start;     ///< [K+1] ranges into pipe_patch
};

constexpr int FUSED_LDS_CELLS = FVHIP_FUSED_ROWS;   ///< staged cells per patch (rows of 112 B), at most
constexpr int FUSED_LDS_CELLS_5W = FVHIP_SLOTS*284/256;   ///< ... for the 5-wave inviscid kernel: 284 x 112 B = 31,808 B, five 256-thread blocks within 160 KB at a 1,280-B allocation granule (FVHIP_SLOTS = 128: ten blocks of 142 rows)
/// the fused kernel's staged-row cap for cfg: 5 blocks of 32 KB per CU for the inviscid unlimited
/// instantiations (compiled for 5 waves per SIMD), else FUSED_LDS_CELLS (4 blocks of 39 KB)
int fusedRowCap(const fvhip_flow_config& cfg);
static_assert(FUSED_LDS_CELLS < 0x8000 && 2*SLOTS_MAX < 0xFFFF, "fused codes are 16-bit");
constexpr int PIPE_CHUNKS = 8;          ///< gradient chunks of the pipelined staged residual

/// whether cfg takes the fused residual kernel (WLS + MUSCL/unlimited linear, inviscid or viscous). On a
/// partitioned mesh, ghost cells in a patch's ring 1 take their received gradients.
bool fusedEligible(const fvhip_flow_config& cfg);
/// builds the fz_* arrays (owned-only meshes)
void buildFused(Layout& Lo);

/// whether cfg takes the pipelined staged residual (order 2, WLS, MUSCL/unlimited linear; viscous
/// allowed) and, if so, builds the pipe_* schedule with `chunks` gradient chunks (single domain)
bool pipelineEligible(const fvhip_flow_config& cfg);
void buildPipeline(Layout& Lo, int chunks);

/// Builds the layout from the reference's mesh arrays. bc_of_tag maps a boundary marker to the
/// index of its BC in the config. Throws std::runtime_error on unsupported meshes.
Layout buildLayout(const fvhip_mesh& m, const fvhip_flow_config& cfg, bool renumber);
struct MeshTopo;
/// Same from a (possibly partitioned) topology: owned cells are renumbered and patched, ghost
/// cells keep internal ids after them and are only read (partition.hpp)
Layout buildLayout(const MeshTopo& T, const fvhip_flow_config& cfg, bool renumber);

}
#endif
