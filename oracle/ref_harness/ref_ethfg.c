/*
 * ref_ethfg.c - flow-group translation unit of the reference harness.
 *
 * TEST INFRASTRUCTURE ONLY. Compiles the reference's dp/core/ethfg.c
 * unmodified (for eth_recv_handle_fg_transition, ethfg.c:502-523, the step
 * that maps a flow-director match's MBUF_INVALID_FG_ID to the CPU's outbound
 * flow group) and supplies link-time doubles for the runtime symbols the rest
 * of that file references. None of the doubles is reached on the path the
 * harness drives (a flow group owned by the current CPU, not in transition).
 */
#include "/root/reference/dp/core/ethfg.c"

#include "ref_capture.h"

/* ---- doubles for ethfg.c's other references (never called here) ---- */
const char __perfg_start[1];
const char __perfg_end[1];
volatile struct cp_shmem *cp_shmem;
DEFINE_PERCPU(volatile struct command_struct *, cp_cmd);
DEFINE_PERCPU(unsigned int, cpu_numa_node);
DEFINE_PERCPU(int, eth_num_queues);
DEFINE_PERCPU(struct eth_rx_queue *, eth_rxqs[NETHDEV]);
void *percpu_offsets[NCPU];
int cpu_run_on_one(cpu_func_t func, void *data, unsigned int cpu)
{
	(void)func;
	(void)data;
	(void)cpu;
	return -1;
}
int eth_process_poll(void) { return 0; }
void *mem_alloc_pages_onnode(int nr, int size, int node, int numa_policy)
{
	(void)nr;
	(void)size;
	(void)node;
	(void)numa_policy;
	return NULL;
}
void mem_free_pages(void *addr, int nr, int size)
{
	(void)addr;
	(void)nr;
	(void)size;
}
void tcp_unified_timer_handler(struct timer *t, struct eth_fg *cur_fg)
{
	(void)t;
	(void)cur_fg;
}
int timer_add(struct timer *t, struct eth_fg *fg, uint64_t usecs)
{
	(void)t;
	(void)fg;
	(void)usecs;
	return 0;
}
int timer_collect_fgs(uint8_t *fg_vector, struct hlist_head *list, uint64_t *timer_pos)
{
	(void)fg_vector;
	(void)list;
	(void)timer_pos;
	return 0;
}
void timer_reinject_fgs(struct hlist_head *list, uint64_t timer_pos)
{
	(void)list;
	(void)timer_pos;
}

/* ---- entry point used by harness_main.c ---- */
static struct eth_fg owned_fg[NCPU]; /* the outbound groups, owned by their CPU */

/* The fg_id eth_recv (inc/ix/ethqueue.h:86-88) leaves in an mbuf whose driver
 * fg_id was `fg_id` (MBUF_INVALID_FG_ID after a flow-director match), on CPU
 * `cpu`; 0xffffffff when the packet would not be processed on this CPU. The
 * groups the mapping can land on are owned by `cpu`. */
uint32_t ref_fg_transition(uint32_t fg_id, unsigned int cpu)
{
	struct mbuf m;
	memset(&m, 0, sizeof(m));
	m.fg_id = (uint16_t)fg_id;
	const unsigned int saved = percpu_get(cpu_id);
	percpu_get(cpu_id) = cpu;
	owned_fg[cpu].cur_cpu = (int)cpu;
	owned_fg[cpu].in_transition = 0;
	struct eth_fg *saved_fg = fgs[ETH_MAX_TOTAL_FG + cpu];
	fgs[ETH_MAX_TOTAL_FG + cpu] = &owned_fg[cpu];
	struct eth_fg *saved_in = fg_id < ETH_MAX_TOTAL_FG + NCPU ? fgs[fg_id] : NULL;
	if (fg_id < ETH_MAX_TOTAL_FG)
		fgs[fg_id] = &owned_fg[cpu];
	const int dropped = eth_recv_handle_fg_transition(NULL, &m);
	if (fg_id < ETH_MAX_TOTAL_FG)
		fgs[fg_id] = saved_in;
	fgs[ETH_MAX_TOTAL_FG + cpu] = saved_fg;
	percpu_get(cpu_id) = saved;
	return dropped ? 0xffffffffu : m.fg_id;
}
