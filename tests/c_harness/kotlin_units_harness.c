/*
 * kotlin_units_harness.c -- drives libinsitu_hip.so's reference-shaped entry points from C, one
 * process per rank, with the argument units the Kotlin host computes (scenery-insitu_amd/jni/
 * kotlin_units.h, the header the JNI adaptor takes its sizes from):
 *
 *   vdi   DistributedVolumes.distributeVDIs(sizePerProcess = H*W*S*4/commSize floats)        :860
 *         -> DistributedVolumeRenderer.gatherCompositedVDIs(subVDILen = H*W*4/commSize bytes) :602
 *   cvdi  DistributedVolumes.distributeVDIs -> DistributedVolumes.gatherCompositedVDIs
 *         (compositedVDILen = H*W*S_out*4/commSize floats)                                    :903
 *   plain DistributedVolumeRenderer.distributeVDIs(sizePerProcess = H*W*4/commSize bytes)    :577
 *         -> gatherCompositedVDIs                                                            :602
 *   frame the device-resident path from C: insitu_set_brick (u16 brick) + insitu_frame
 *   ktgrids / ktplain  DistributedVolumeRenderer's device-resident frame with the Kotlin arguments
 *         (jni/kotlin_device_path.h, the bodies of the JNI externals insituUpdateData + insituFrame):
 *         updateData's grid arrays (origins, gridDims, pixelToWorld) -> kt_update_data, kt_frame; VDI
 *         flatten or plain mode, image to the root as streamImage receives it
 *   ktpipe    as ktgrids through insituFramePipelined + insituFrameFlush (kt_frame_pipelined, kt_frame_flush):
 *         two frames of the same camera, both images written (image0.bin, image.bin)
 *   ktvolume  DistributedVolumes' (insituUpdateVolume + insituFrame): kt_update_volume, kt_frame, the
 *         gathered composited VDI read where gatherCompositedVDIs leaves it
 *
 * usage: kotlin_units_harness --abi
 *        kotlin_units_harness <vdi|cvdi|plain|frame|ktgrids|ktpipe|ktplain|ktvolume> <dir> <rank> <nranks> <device>
 * <dir>/case.txt holds "W H S S_out nx ny nz"; inputs are raw files written by
 * tests/test_c_harness.py (camera.bin = struct insitu_camera, tf.bin, cmap.bin, sub_col_<r>.bin,
 * sub_dep_<r>.bin, brick_<r>.bin, model_<r>.bin; the kt kinds: grid_<r>.bin u16 voxels, origins_<r>.bin /
 * griddims_<r>.bin int32 (3 / 6 per grid), pos_<r>.bin float32 x3, p2w.bin float32).  Rank 0 creates the ncclUniqueId and publishes it
 * as <dir>/commid.bin; outputs: recv_col_<r>.bin, recv_dep_<r>.bin, and on rank 0 image.bin or
 * gcol.bin / gdep.bin.  Exit status 0 = every call returned 0.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "insitu_hip.h"
#include "kotlin_device_path.h"
#include "kotlin_units.h"

static char g_dir[4096];

static void die(insitu_ctx* c, const char* what) {
    fprintf(stderr, "harness: %s failed: %s\n", what, insitu_last_error(c));
    exit(1);
}

static void* read_file(const char* name, long long* bytes) {
    char path[4200];
    snprintf(path, sizeof path, "%s/%s", g_dir, name);
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "harness: cannot open %s\n", path); exit(1); }
    fseek(f, 0, SEEK_END);
    long long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* p = malloc(n > 0 ? (size_t)n : 1);
    if (n > 0 && fread(p, 1, (size_t)n, f) != (size_t)n) { fprintf(stderr, "harness: short read %s\n", path); exit(1); }
    fclose(f);
    if (bytes) *bytes = n;
    return p;
}

static void write_file(const char* name, const void* p, long long bytes) {
    char path[4200], tmp[4300];
    snprintf(path, sizeof path, "%s/%s", g_dir, name);
    snprintf(tmp, sizeof tmp, "%s.tmp", path);
    FILE* f = fopen(tmp, "wb");
    if (!f || fwrite(p, 1, (size_t)bytes, f) != (size_t)bytes) { fprintf(stderr, "harness: cannot write %s\n", tmp); exit(1); }
    fclose(f);
    if (rename(tmp, path) != 0) { fprintf(stderr, "harness: rename %s\n", path); exit(1); }
}

static void need_size(const char* what, long long got, long long want) {
    if (got != want) { fprintf(stderr, "harness: %s has %lld bytes, expected %lld\n", what, got, want); exit(1); }
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "--abi") == 0) {
        printf("insitu_abi_version %d\n", insitu_abi_version());
        return insitu_abi_version() == INSITU_ABI_VERSION ? 0 : 1;
    }
    if (argc != 6) {
        fprintf(stderr, "usage: %s --abi | <vdi|cvdi|plain|frame|ktgrids|ktpipe|ktplain|ktvolume> <dir> <rank> <nranks> <device>\n", argv[0]);
        return 2;
    }
    const char* kind = argv[1];
    snprintf(g_dir, sizeof g_dir, "%s", argv[2]);
    const int rank = atoi(argv[3]), nranks = atoi(argv[4]), device = atoi(argv[5]);
    const int vdi = strcmp(kind, "plain") != 0 && strcmp(kind, "ktplain") != 0;
    const int cvdi = strcmp(kind, "cvdi") == 0 || strcmp(kind, "ktvolume") == 0;
    const int frame = strcmp(kind, "frame") == 0;
    const int kt = strncmp(kind, "kt", 2) == 0;
    int W, H, S, S_out, dims[3];
    {
        long long n;
        char* txt = (char*)read_file("case.txt", &n);
        txt = (char*)realloc(txt, (size_t)n + 1);
        txt[n] = 0;
        if (sscanf(txt, "%d %d %d %d %d %d %d", &W, &H, &S, &S_out, &dims[0], &dims[1], &dims[2]) != 7) {
            fprintf(stderr, "harness: bad case.txt\n");
            return 2;
        }
        free(txt);
    }

    /* the ncclUniqueId: created on rank 0, published through the directory (the simulation's
       MPI_Bcast in a real deployment) */
    unsigned char comm_id[INSITU_COMM_ID_BYTES];
    if (nranks > 1) {
        char path[4200];
        snprintf(path, sizeof path, "%s/commid.bin", g_dir);
        if (rank == 0) {
            if (insitu_comm_id(comm_id, sizeof comm_id) != 0) die(NULL, "insitu_comm_id");
            write_file("commid.bin", comm_id, sizeof comm_id);
        } else {
            int waited = 0;
            while (access(path, R_OK) != 0) {
                if (++waited > 12000) { fprintf(stderr, "harness: no commid.bin\n"); return 1; }
                usleep(10000);
            }
            long long n;
            void* p = read_file("commid.bin", &n);
            need_size("commid.bin", n, sizeof comm_id);
            memcpy(comm_id, p, sizeof comm_id);
            free(p);
        }
    }

    insitu_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.rank = rank;
    cfg.nranks = nranks;
    cfg.device = device;
    cfg.width = W;
    cfg.height = H;
    cfg.max_supersegments = vdi ? S : 1;
    cfg.mode = vdi ? INSITU_MODE_VDI : INSITU_MODE_PLAIN;
    cfg.bricks_per_rank = 1;
    cfg.comm_id = nranks > 1 ? comm_id : NULL;
    cfg.composite_vdi = cvdi;
    cfg.max_output_supersegments = cvdi ? S_out : 0;
    insitu_ctx* ctx = NULL;
    if (insitu_create(&cfg, &ctx) != 0) die(NULL, "insitu_create");

    long long n;
    insitu_camera* cam = (insitu_camera*)read_file("camera.bin", &n);
    need_size("camera.bin", n, sizeof(insitu_camera));
    long long ntf, ncm;
    float* tf = (float*)read_file("tf.bin", &ntf);
    float* cmap = (float*)read_file("cmap.bin", &ncm);
    float conv[2] = {1.0f, 0.0f};
    {
        long long nc;
        float* cv = (float*)read_file("conv.bin", &nc);
        need_size("conv.bin", nc, sizeof conv);
        memcpy(conv, cv, sizeof conv);
        free(cv);
    }
    if (insitu_set_transfer(ctx, tf, (int)(ntf / 4), cmap, (int)(ncm / 16), conv[0], conv[1]) != 0)
        die(ctx, "insitu_set_transfer");

    char name[64];
    if (kt) {   /* the Kotlin device-resident frame (kotlin_device_path.h, as the JNI externals run it) */
        long long pn;
        float* p2w = (float*)read_file("p2w.bin", &pn);
        need_size("p2w.bin", pn, 4);
        snprintf(name, sizeof name, "grid_%d.bin", rank);
        void* grid = read_file(name, &n);
        need_size(name, n, (long long)dims[0] * dims[1] * dims[2] * 2);
        if (strcmp(kind, "ktvolume") == 0) {   /* insituUpdateVolume(volumeID 0, buffer, dims, pos, is16bit) */
            snprintf(name, sizeof name, "pos_%d.bin", rank);
            float* pos = (float*)read_file(name, &n);
            need_size(name, n, 12);
            if (kt_update_volume(ctx, 0, grid, 0, dims, 1, pos, *p2w) != 0) die(ctx, "kt_update_volume");
            if (kt_frame(ctx, cam->view, cam->proj, cam->inv_view, cam->inv_proj, cam->nw, 0.0f, NULL, 0) != 0)
                die(ctx, "kt_frame");
            if (rank == 0) {   /* gatherColorPointer / gatherDepthPointer */
                const size_t cb = insitu_buffer_bytes(ctx, INSITU_BUF_GATHERED_COLOR);
                const size_t db = insitu_buffer_bytes(ctx, INSITU_BUF_GATHERED_DEPTH);
                void* gc = malloc(cb);
                void* gd = malloc(db);
                if (insitu_read(ctx, INSITU_BUF_GATHERED_COLOR, 0, gc, cb) != 0) die(ctx, "insitu_read gathered colour");
                if (insitu_read(ctx, INSITU_BUF_GATHERED_DEPTH, 0, gd, db) != 0) die(ctx, "insitu_read gathered depth");
                write_file("gcol.bin", gc, (long long)cb);
                write_file("gdep.bin", gd, (long long)db);
            }
        } else {   /* insituUpdateData(1 grid) + insituFrame -> streamImage on the root */
            snprintf(name, sizeof name, "origins_%d.bin", rank);
            int* origins = (int*)read_file(name, &n);
            need_size(name, n, 12);
            snprintf(name, sizeof name, "griddims_%d.bin", rank);
            int* gdims = (int*)read_file(name, &n);
            need_size(name, n, 24);
            const void* grids[1] = {grid};
            if (kt_update_data(ctx, 1, grids, 0, origins, gdims, *p2w) != 0) die(ctx, "kt_update_data");
            const size_t cap = insitu_buffer_bytes(ctx, INSITU_BUF_IMAGE);
            unsigned char* img = cap ? (unsigned char*)malloc(cap) : NULL;
            if (strcmp(kind, "ktpipe") == 0) {   /* insituFramePipelined twice (the same camera) + insituFrameFlush */
                long long done = 0;
                if (kt_frame_pipelined(ctx, cam->view, cam->proj, cam->inv_view, cam->inv_proj, cam->nw, cam->fwnw, img,
                                       cap, &done) != 0 || done != -1)
                    die(ctx, "kt_frame_pipelined (first call)");
                if (kt_frame_pipelined(ctx, cam->view, cam->proj, cam->inv_view, cam->inv_proj, cam->nw, cam->fwnw, img,
                                       cap, &done) != 0 || done != 0)
                    die(ctx, "kt_frame_pipelined (second call)");
                if (rank == 0) write_file("image0.bin", img, (long long)cap);
                if (kt_frame_flush(ctx, img, cap, &done) != 0 || done != 1) die(ctx, "kt_frame_flush");
            } else if (kt_frame(ctx, cam->view, cam->proj, cam->inv_view, cam->inv_proj, cam->nw, cam->fwnw, img, cap) != 0) {
                die(ctx, "kt_frame");
            }
            if (rank == 0) write_file("image.bin", img, (long long)cap);
        }
        insitu_destroy(ctx);
        printf("HARNESS_OK %s rank %d\n", kind, rank);
        return 0;
    }
    if (frame) {   /* device-resident path: brick upload + whole frame */
        snprintf(name, sizeof name, "brick_%d.bin", rank);
        void* brick = read_file(name, &n);
        need_size(name, n, (long long)dims[0] * dims[1] * dims[2] * 2);
        snprintf(name, sizeof name, "model_%d.bin", rank);
        float* model = (float*)read_file(name, &n);
        need_size(name, n, 64);
        if (insitu_set_brick(ctx, 0, brick, INSITU_U16, dims, model, 0) != 0) die(ctx, "insitu_set_brick");
        const size_t cap = (size_t)W * H * 4;
        unsigned char* img = rank == 0 ? (unsigned char*)malloc(cap) : NULL;
        if (insitu_frame(ctx, cam, img, cap) != 0) die(ctx, "insitu_frame");
        if (rank == 0) write_file("image.bin", img, (long long)cap);
        insitu_destroy(ctx);
        printf("HARNESS_OK frame rank %d\n", rank);
        return 0;
    }

    if (insitu_set_camera(ctx, cam) != 0) die(ctx, "insitu_set_camera");
    const long long spp = kt_size_per_process(W, H, vdi ? S : 1, nranks);
    snprintf(name, sizeof name, "sub_col_%d.bin", rank);
    void* col = read_file(name, &n);
    need_size(name, n, kt_recv_colour_bytes(vdi, spp, nranks));   /* a sub-VDI is commSize blocks */
    snprintf(name, sizeof name, "sub_dep_%d.bin", rank);
    void* dep = read_file(name, &n);
    need_size(name, n, kt_recv_depth_bytes(vdi, spp, nranks));
    const long long rcb = kt_recv_colour_bytes(vdi, spp, nranks), rdb = kt_recv_depth_bytes(vdi, spp, nranks);
    void* rcol = malloc((size_t)rcb);
    void* rdep = malloc((size_t)rdb);
    if (insitu_distribute_vdis(ctx, col, dep, spp, nranks, rcol, rdep) != 0) die(ctx, "insitu_distribute_vdis");
    snprintf(name, sizeof name, "recv_col_%d.bin", rank);
    write_file(name, rcol, rcb);
    snprintf(name, sizeof name, "recv_dep_%d.bin", rank);
    write_file(name, rdep, rdb);

    if (cvdi) {
        const long long len = kt_gather_len(W, H, S_out, 1, nranks);
        const long long gcb = kt_gather_colour_bytes(len, nranks), gdb = kt_gather_depth_bytes(len, nranks);
        void* gc = rank == 0 ? malloc((size_t)gcb) : NULL;
        void* gd = rank == 0 ? malloc((size_t)gdb) : NULL;
        if (insitu_gather_composited_vdi_set(ctx, len, 0, rank, nranks, gc, gd) != 0)
            die(ctx, "insitu_gather_composited_vdi_set");
        if (rank == 0) {
            write_file("gcol.bin", gc, gcb);
            write_file("gdep.bin", gd, gdb);
        }
    } else {
        const long long len = kt_gather_len(W, H, 1, 1, nranks);   /* rgba8 bytes per rank */
        const size_t cap = (size_t)(len * nranks);
        unsigned char* img = rank == 0 ? (unsigned char*)malloc(cap) : NULL;
        if (insitu_gather_composited_vdis(ctx, 0, len, rank, nranks, img, cap) != 0)
            die(ctx, "insitu_gather_composited_vdis");
        if (rank == 0) write_file("image.bin", img, (long long)cap);
    }
    insitu_destroy(ctx);
    printf("HARNESS_OK %s rank %d\n", kind, rank);
    return 0;
}
