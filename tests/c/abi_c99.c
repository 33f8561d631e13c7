/* Compiled as C99 by tests/test_abi.py: include/hsflow.h is a plain C
 * header (no C++ constructs outside __cplusplus) and libhsflow.so links
 * and answers the GPU-free entry points from C. */
#include <stdio.h>
#include <string.h>

#include "hsflow.h"

int main(void) {
    int bad = 0;
    if (hsflow_version() != HSFLOW_VERSION) bad |= 1;
    if (strcmp(hsflow_status_string(HSFLOW_ERR_SIZE), "image sizes differ") != 0) bad |= 2;
    if (hsflow_workspace_bytes(1080, 1920, 2) < (size_t)1080 * 1920 * 2 * 24) bad |= 4;
    int r = 0, c = 0;
    if (hsflow_pyramid_level_size(4320, 7680, 2, &r, &c) != HSFLOW_OK || r != 1080 || c != 1920)
        bad |= 8;
    unsigned char bgr[6] = {10, 20, 30, 200, 100, 0}, gray[2];
    if (hsflow_bgr_to_gray(bgr, 1, 2, 6, gray, 2) != HSFLOW_OK) bad |= 16;
    /* argument validation happens before any device work */
    if (hsflow_flow_device(NULL, NULL, HSFLOW_U8, 8, 8, 1, 5, 1, 1.0f, NULL, NULL, NULL, 0,
                           NULL) != HSFLOW_ERR_ARG)
        bad |= 32;
    printf("%d %u %u\n", bad, gray[0], gray[1]);
    return bad;
}
